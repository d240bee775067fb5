"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs, gpurun_out/pmc_traffic/*) into
bench_pmc_traffic.json: per kernel family, the average HBM bytes per launch corrected as
MI355X_MICROARCH.md prescribes (2 x FETCH_SIZE + WRITE_SIZE, counters in KiB).
Usage: python scripts/pmc_traffic.py <dir with f32_fetch/f32_write/bf16_fetch/bf16_write csvs>
       python scripts/pmc_traffic.py --gemm <dir with fetch/write csvs of scripts/gemm_traffic.py>"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAMILIES = {  # json key -> kernel-name prefix
    "lstm_step_bwd_v2_kernel": "void lstm_step_bwd_v2_kernel<",
    "lstm_step_fwd_v2_kernel": "void lstm_step_fwd_v2_kernel<32, 101",
    "lstm_persist2_bwd_bf16_kernel": "void lstm_persist2_bwd_bf16_kernel<",
    "lstm_persist2_fwd_bf16_kernel": "void lstm_persist2_fwd_bf16_kernel<48, 32, 0>",  # (c5 rank: 32 x 32 tiles)
    "lstm_persist3_bwd_bf16_kernel": "void lstm_persist3_bwd_bf16_kernel<",
    "lstm_persist3_fwd_bf16_kernel": "void lstm_persist3_fwd_bf16_kernel<",
    "lstm_persist_bwd_f32_h2_kernel": "void lstm_persist_bwd_f32_h2_kernel<",
    "lstm_persist_fwd_f32_kernel": "void lstm_persist_fwd_f32_kernel<",
    # the rank shapes (scripts/persist_ab.py passes c4: B = 80, T = 160; c5: B = 320, T = 180)
    "lstm_wave3_fwd_bf16_kernel": "void lstm_wave3_fwd_bf16_kernel<",
    "lstm_wave_bwd_bf16_kernel": "void lstm_wave_bwd_bf16_kernel<",
    "gemm_bf16_8qf_kernel@c4": "(anonymous namespace)::gemm_bf16_8qf_kernel",
    # in-step GEMMs, per shape (c2 fp32 / c3 bf16, B = 640, T = 160, H = 768): (prefix, grid threads)
    # (r04 names: the K1 is the persistent 256p kernel, the dx GEMM reads the fragment-order A (AF = 1),
    # the dW GEMMs are split-K slabs (EPI = 1); the template's 4th argument is AF)
    "gemm_f32_256p_kernel<256,32>@K1.in_step": "void gemm_f32_256p_kernel<256, 32>",
    "gemm_f32_256sk_kernel<256,1>@dx.in_step": "void gemm_f32_256sk_kernel<256, 1>",  # stream-K dx (r04)
    "gemm_f32_256_kernel<256,32,1,0>@dW.in_step": "void gemm_f32_256_kernel<256, 32, 1, 0>",
    "gemm_bf16_8qp_kernel<2>@K1.in_step": "void gemm_bf16_8qp_kernel<2>",
    "gemm_bf16_8q_kernel<0,1>@dx.in_step": "void gemm_bf16_8q_kernel<0, 1>",
    "gemm_bf16_8q_kernel<1,0>@dW.in_step": "void gemm_bf16_8q_kernel<1, 0>",
}
B_, T_, H_ = 640, 160, 768
# scripts/gemm_traffic.py's isolated launches: key -> (prefix, grid or None, algorithmic bytes)
GEMM = {
    "gemm_f32_256_kernel<256,32,0>": ("void gemm_f32_256_kernel<256, 32, 0>", 400 * 12 * 512,
                                      4 * (T_ * B_ * H_ + 4 * H_ * H_ + T_ * B_ * 4 * H_)),
    "gemm_f32_256_kernel<256,32,0>@dx": ("void gemm_f32_256_kernel<256, 32, 0>", 400 * 3 * 512,
                                         4 * (T_ * B_ * 4 * H_ + 4 * H_ * H_ + T_ * B_ * H_)),
    "gemm_f32_256_kernel<256,32,1>@dW": ("void gemm_f32_256_kernel<256, 32, 1>", None,
                                         4 * (T_ * B_ * 4 * H_ + T_ * B_ * H_ + 4 * H_ * H_)),
    # the persistent fp32 NT GEMM (one workgroup per CU: K1 and dx have the same grid) -- told apart
    # by launch order: gemm_traffic.py runs 1 + REPS launches of K1 (Gx), later 1 + REPS of dx
    "gemm_f32_256p_kernel<256,32>@K1": ("void gemm_f32_256p_kernel<256, 32>", None,
                                        4 * (T_ * B_ * H_ + 4 * H_ * H_ + T_ * B_ * 4 * H_), (0, 4)),
    "gemm_f32_256p_kernel<256,32>@dx": ("void gemm_f32_256p_kernel<256, 32>", None,
                                        4 * (T_ * B_ * 4 * H_ + 4 * H_ * H_ + T_ * B_ * H_), (4, 8)),
    "gemm_bf16_8qp_kernel<2>@K1": ("void gemm_bf16_8qp_kernel<2>", None,
                                   2 * (T_ * B_ * H_ + 4 * H_ * H_ + T_ * B_ * 4 * H_)),
    "gemm_bf16_8q_kernel<0,0>@dx": ("void gemm_bf16_8q_kernel<0, 0>", None,
                                    2 * (T_ * B_ * 4 * H_ + 4 * H_ * H_) + 4 * T_ * B_ * H_),
    "gemm_bf16_8q_kernel<1,0>@dW": ("void gemm_bf16_8q_kernel<1, 0>", None,
                                    2 * (T_ * B_ * 4 * H_ + T_ * B_ * H_) + 4 * 4 * H_ * H_),
}


def _grid(r):
    for c in ("Grid_Size", "Grid_Size_X"):
        if r.get(c):
            return int(r[c])
    return None


def per_launch(path, counter, families):
    """Average counter value per launch of each family; a spec's optional 4th item (lo, hi) keeps only
    the family's matching launches lo .. hi - 1 in dispatch order."""
    acc, seen = {}, {}
    rows = list(csv.DictReader(open(path)))
    if rows and "Dispatch_Id" in rows[0]:
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        for key, spec in families.items():
            pre, grid = (spec, None) if isinstance(spec, str) else spec[:2]
            if r["Kernel_Name"].startswith(pre) and (grid is None or _grid(r) == grid):
                i = seen.get(pre, 0) if len(spec) > 3 and not isinstance(spec, str) else None
                if i is not None and not (spec[3][0] <= i < spec[3][1]):
                    continue
                s, n = acc.get(key, (0.0, 0))
                acc[key] = (s + float(r["Counter_Value"]), n + 1)
        for pre in {(sp if isinstance(sp, str) else sp[0]) for sp in families.values()}:
            if r["Kernel_Name"].startswith(pre):
                seen[pre] = seen.get(pre, 0) + 1
    return {k: s / n for k, (s, n) in acc.items()}


def gemm_main(d, data):
    fs = glob.glob(os.path.join(d, "fetch*", "**", "*counter_collection.csv"), recursive=True)
    ws = glob.glob(os.path.join(d, "write*", "**", "*counter_collection.csv"), recursive=True)
    fetch, write = per_launch(fs[0], "FETCH_SIZE", GEMM), per_launch(ws[0], "WRITE_SIZE", GEMM)
    for k, spec in GEMM.items():
        alg = spec[2]
        if k in fetch and k in write:
            hbm = int(1024 * (2 * fetch[k] + write[k]))
            data[k] = {"FETCH_SIZE_KiB": round(fetch[k], 1), "WRITE_SIZE_KiB": round(write[k], 1),
                       "hbm_bytes_per_launch": hbm, "algorithmic_bytes": alg, "ratio": round(hbm / alg, 3),
                       "source": "rocprofv3 --pmc over scripts/gemm_traffic.py (isolated launches, c2/c3 shapes)"}


def main(d, gemm=False):
    out_path = os.path.join(ROOT, "bench_pmc_traffic.json")  # read by bench.py (profiles/ stays here)
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data.pop("gemm_f32_256_kernel<256,32,0,1>@dx.in_step", None)  # the one-shot dx, replaced in-step by stream-K
    if gemm:
        gemm_main(d, data)
    for tag in () if gemm else ("f32", "bf16", "c4", "c5"):
        fs = glob.glob(os.path.join(d, f"{tag}_fetch*", "**", "*counter_collection.csv"), recursive=True)
        ws = glob.glob(os.path.join(d, f"{tag}_write*", "**", "*counter_collection.csv"), recursive=True)
        if not fs or not ws:
            continue
        fetch, write = per_launch(fs[0], "FETCH_SIZE", FAMILIES), per_launch(ws[0], "WRITE_SIZE", FAMILIES)
        for k0 in fetch:
            if k0 not in write:
                continue
            # the rank passes' GEMMs (other shapes than c2 / c3's) under their own keys
            k = f"{tag}:{k0}" if tag in ("c4", "c5") and "@" in k0 and not k0.endswith("@c4") else k0
            if True:
                data[k] = {"FETCH_SIZE_KiB": round(fetch[k0], 1), "WRITE_SIZE_KiB": round(write[k0], 1),
                           "hbm_bytes_per_launch": int(1024 * (2 * fetch[k0] + write[k0])),
                           "source": f"rocprofv3 --pmc over {'bench.py' if tag in ('f32', 'bf16') else 'scripts/persist_ab.py'} "
                                     f"({tag} step, in-step launches; "
                                     f"{os.path.basename(os.path.normpath(os.path.join(d, '..')))})"}
    data["_note"] = ("rocprofv3 --pmc passes, FETCH_SIZE and WRITE_SIZE in separate runs; hbm_bytes = 2*FETCH_SIZE + "
                     "WRITE_SIZE (gfx950 halves wide reads, MI355X_MICROARCH.md §HBM); FETCH_SIZE counts L2 misses "
                     "incl. Infinity-Cache hits.  In-step entries: scripts/gpu_pmc_traffic.sh + scripts/pmc_traffic.py")
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in data.items() if isinstance(v, dict)}))


if __name__ == "__main__":
    if sys.argv[1] == "--gemm":
        main(sys.argv[2], gemm=True)
    else:
        main(sys.argv[1])
