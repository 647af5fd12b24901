"""irlmx_dense_gemm (the hand-written fp64 MFMA kernel, dense.hip) at S = 4096
with B = 16 and B = 64, ten launches each after a warm-up, for a rocprofv3
--kernel-trace --stats pass; prints the HIP-event average per launch too."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import ops
dev = torch.device("cuda", 0)
for S, B in ((4096, 16), (4096, 64), (2048, 16), (2048, 64)):
    g = torch.Generator(device=dev).manual_seed(S + B)
    m = torch.rand((S, S), dtype=torch.float64, device=dev, generator=g)
    z = torch.rand((B, S), dtype=torch.float64, device=dev, generator=g)
    ops.dense_gemm(m, z)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.dense_gemm(m, z)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100.0
    print(f"S={S} B={B} variant={ops.dense_gemm_variant(S, S, B)} {us:.1f} us/launch "
          f"{2.0 * S * S * B / us / 1e6:.2f} TFLOP/s")
