#!/bin/bash
# iteration: fp32 model tests + a short c2 bench (no extras)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out
T=${TAG:-f1}
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_status.py -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pt_$T.log 2>&1
rc=$?; grep -E "MEASURED|passed|failed|Error" gpurun_out/pt_$T.log | tail -24
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vendor --no-f32x --no-extras --no-bf16 > gpurun_out/bench_$T.log 2>&1; rc=$?
python - <<'PY'
import json,os
t=os.environ.get("TAG","f1")
l=[x for x in open(f"gpurun_out/bench_{t}.log") if x.startswith("{")]
d=json.loads(l[-1]); print("c2", d["ms_per_step"], "ms", d["value"], d["roofline"]["frac"], d.get("roofline_fwd",{}).get("frac"))
PY
exit $rc
