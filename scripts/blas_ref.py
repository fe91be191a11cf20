"""Library bar for the tower GEMMs: torch.nn.functional.linear (hipBLASLt on
ROCm) on the scripts/gemm_micro.py shapes, random bf16, HIP events.
usage: python scripts/blas_ref.py [reps]"""
import sys

import torch

SHAPES = {"qkv": (100000, 2304, 768), "out": (100000, 768, 768), "fc": (100000, 3072, 768),
          "proj": (100000, 768, 3072), "long": (16384, 4096, 4096),
          # the bench's 500k-row pass (10k ViT-B/32 frames): the library's plain bf16 GEMM + bias at
          # the shapes of the tower's LN-folded / fused kernels
          "qkv500": (500000, 2304, 768), "out500": (500000, 768, 768), "fc500": (500000, 3072, 768),
          "proj500": (500000, 768, 3072)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    for name, (M, N, K) in SHAPES.items():
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).bfloat16()
        b = torch.rand(N, device=dev).bfloat16()
        torch.nn.functional.linear(A, W, b)
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                torch.nn.functional.linear(A, W, b)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
        print(f"hipblaslt {name:5s} M={M} N={N} K={K}: {best:9.1f} us {2.0 * M * N * K / best / 1e6:7.1f} TFLOP/s",
              flush=True)


if __name__ == "__main__":
    main()
