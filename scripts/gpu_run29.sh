#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r29
timeout -k 10 400 python -u -m pytest tests/test_dvector.py tests/test_gpu_dropin_cpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r29/pt.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r29/pt.log; exit 1; }
grep -E "MEASURED graphed_f32|passed|failed" gpurun_out/r29/pt.log
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda', 0)
net, _ = bench.build_model(bench.DIMS, dev)
print(json.dumps(bench.dvector_inference(net, dev)['per_file_call']))
" > gpurun_out/r29/dvec.log 2>&1 || { echo "dvec rc=$?"; tail -20 gpurun_out/r29/dvec.log; exit 1; }
tail -1 gpurun_out/r29/dvec.log
