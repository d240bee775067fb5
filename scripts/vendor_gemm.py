"""Times the vendor bf16 GEMM (torch.matmul -> hipBLASLt) at the c3 step's GEMM shapes, for
comparison with the in-step kernels (K1 input projection, dx, the dual dW).  Prints one JSON line
per shape: ms per call and TFLOP/s."""
import json

import torch


def timed(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda:0")
    TB, H, G = 160 * 640, 768, 3072
    shapes = {  # name: (M, N, K)
        "K1 gates = h W_ih^T": (TB, G, H),
        "dx = dG W_ih": (TB, H, G),
        "dual dW = dG^T [x; h]": (G, 2 * H, TB),
    }
    for name, (M, N, K) in shapes.items():
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        bt = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        ms = timed(lambda: torch.matmul(a, bt.t()))
        ms32 = None
        try:
            out = torch.empty(M, N, device=dev, dtype=torch.float32)
            ms32 = timed(lambda: torch.mm(a, bt.t(), out_dtype=torch.float32, out=out))
        except Exception as ex:  # out_dtype needs a recent torch
            ms32 = f"{type(ex).__name__}"
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "ms_bf16_out": round(ms, 4),
                          "tflops": round(2 * M * N * K / ms / 1e9, 1), "ms_f32_out": ms32}), flush=True)
        del a, bt


if __name__ == "__main__":
    main()
