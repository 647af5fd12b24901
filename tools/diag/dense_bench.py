"""Dense-row path timings (IRLMX_LAYOUT_DENSE): per-sweep cost of the backward
(streaming M once per instance on the VALU vs one fp64-MFMA GEMM over all B
instances of a shared table), the forward, soft VI and VI, on random dense
tables.  usage: python tools/diag/dense_bench.py [S ...]
(round 2 also timed a rocBLAS dgemm here; round 3 removed the library)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import numpy as np, torch
from irlmx import DeviceMDP, ops
from irlmx.batch import terminal_reward

dev = torch.device("cuda", 0)
sizes = [int(a) for a in sys.argv[1:]] or [2048, 4096]
for S in sizes:
    rng = np.random.default_rng(S)
    P = rng.random((S, S, 4)) + 1e-3
    P /= P.sum(axis=1, keepdims=True)
    one = DeviceMDP.from_dense(P, device=dev)
    del P
    for B in [int(x) for x in os.environ.get("BATCHES", "1,4,16,64").split(",")]:
        mdp = one.with_batch(B)
        r = rng.uniform(0.0, 1.0, (B, S))
        tm = ops.terminal_mask([S - 1], S, batch=B, device=dev)
        res = {}
        for mode, env in (("stream", "1000000"), ("gemm-mfma", "1")):
            if B == 1 and mode != "stream":
                continue
            if os.environ.get("MODES") and mode not in os.environ["MODES"].split(","):
                continue
            os.environ["IRLMX_DENSE_GEMM_MIN"] = env
            ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
            t = time.perf_counter(); pi = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
            dt = time.perf_counter() - t
            res[mode] = dt
            print(f"S={S} B={B} backward {mode}: {dt * 1e3:.1f} ms = {dt / (2 * S) * 1e6:.2f} us/sweep, "
                  f"{B * S * S * 8 * 2 * S / dt / 1e9 if mode == 'stream' else S * S * 8 * 2 * S / dt / 1e9:.0f} GB/s "
                  f"matrix stream, {2.0 * S * S * B * 2 * S / dt / 1e12:.2f} TFLOP/s", flush=True)
        os.environ.pop("IRLMX_DENSE_GEMM_MIN", None)
        if B in (1, 16) and not os.environ.get("BACKWARD_ONLY"):
            pi = ops.backward_maxent(mdp, r, tm)
            p0 = np.zeros((B, S)); p0[:, 0] = 1.0
            torch.cuda.synchronize(); t = time.perf_counter()
            svf, k, _ = ops.forward_svf(mdp, p0, tm, pi); torch.cuda.synchronize(); dt = time.perf_counter() - t
            kk = int(k.max())
            print(f"S={S} B={B} forward: {kk} sweeps {dt * 1e3:.1f} ms = {dt / kk * 1e6:.2f} us/sweep, "
                  f"{B * S * S * 8 * kk / dt / 1e9:.0f} GB/s", flush=True)
            phi = terminal_reward([S - 1], S, B, dev)
            torch.cuda.synchronize(); t = time.perf_counter()
            _, _, ks, _ = ops.soft_backward(mdp, r, phi, 0.7); torch.cuda.synchronize(); dt = time.perf_counter() - t
            kk = int(ks.max())
            print(f"S={S} B={B} soft VI: {kk} sweeps {dt * 1e3:.1f} ms = {dt / kk * 1e6:.2f} us/sweep, "
                  f"{B * 4 * S * S * 8 * kk / dt / 1e9:.0f} GB/s", flush=True)
