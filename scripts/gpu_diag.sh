#!/bin/bash
# fp32 persistent forward graph-replay diagnostic (scripts/f32_replay_diag.py) over A/B builds,
# then the regression / new GPU tests on the product library
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-r405}; mkdir -p $O
run() { echo "== $*" >> $O/diag.log; timeout -k 10 240 python -u scripts/f32_replay_diag.py "$@" >> $O/diag.log 2>&1 || { echo "diag $* rc=$?"; tail -20 $O/diag.log; exit 1; }; }
run --phase B --reps 4 --between none --lib scripts/ab/libsv_ge2e_chk.so
run --phase AB --reps 2 --lib scripts/ab/libsv_ge2e_memset.so
run --phase AB --reps 2
grep -E "^==|phase|memset|emb_vs" $O/diag.log | sed -e 's/"first": {[^}]*}/F/' | cut -c1-300
timeout -k 10 900 python -u -m pytest tests/test_dvector.py tests/test_gpu_sharded.py tests/test_gpu_dp.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "MEASURED|PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -40
exit $rc
