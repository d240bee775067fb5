#!/bin/bash
# A/B: persistent backward recurrences with / without the operand-prefetch helper workgroups
# (bf16 c3: persist_ab.py; fp32 c2: f32_step_ab.py); then the bench (no extras) and parity tests
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-r411}; mkdir -p $O
for r in 1 2 3; do
for v in prod p3pf; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/bf16.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/bf16.log; exit 1; }
done
for v in nopf prod; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --iters 3 --only persist >> $O/f32.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/f32.log; exit 1; }
done
done
grep '"B"' $O/f32.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); p = d['persist']
    print(d['lib'].split('/')[-1], p['fwd_ms'], p['bwd_ms'], p['step_ms'], p['bwd_layer_us'])"
grep '^{' $O/bf16.log | cut -c1-200
timeout -k 10 200 python -u scripts/wave_stamps.py --lib scripts/ab/libsv_ge2e_wst.so > $O/wave.log 2>&1 || { echo "wave rc=$?"; tail -5 $O/wave.log; exit 1; }
grep '^{' $O/wave.log
timeout -k 10 300 python -u bench.py --no-f32x --no-extras --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); print('c2', d['ms_per_step'], d['roofline']['frac'], 'c3', d['bf16']['ms_per_step'], d['roofline_bf16']['frac'], d['roofline_bf16_fwd']['frac'], 'c4r', d['c4_rank_shape']['ms_per_step'], 'c5r', d['c5_rank_shape']['ms_per_step'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_status.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "MEASURED c3|passed|failed" $O/pytest.log | tail -10
exit $rc
