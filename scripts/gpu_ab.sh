#!/bin/bash
# A/B bench runs over env settings: AB_ENVS="VAR=a VAR=b,VAR2=c ..." (one short bench per
# setting; commas join several variables into one setting).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kv in ${AB_ENVS}; do
  env ${kv//,/ } timeout -k 10 300 python bench.py --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab_$kv.log 2>&1 || { echo "ab $kv failed"; tail -5 gpurun_out/ab_$kv.log; exit 1; }
  python3 - "$kv" gpurun_out/ab_$kv.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
r = d.get("roofline", {})
extra = {k: d[k]["ms_per_step"] for k in ("bf16", "c4_rank_shape", "c5_rank_shape", "f32_bf16x6") if k in d}
rb = d.get("roofline_bf16") or {}
print(sys.argv[1], "ms/step", d["ms_per_step"], "roofline", r.get("avg_launch_us"), r.get("frac"), extra,
      "bf16 roof", rb.get("avg_launch_us"), d.get("roofline_fwd", d.get("roofline_bf16_fwd", {})).get("avg_launch_us"))
PY
done
