#!/usr/bin/env python
"""Benchmark: batched MaxEnt-IRL gradient steps on MI355X.

Metric (BASELINE.json): IRL gradient steps/sec (VI + SVF sweep), NxN grid, batch B.
One "step" = one gradient step of maxent.irl (maxent.py:240-252) for every
instance of the batch: backward pass (2*S sweeps) + forward SVF pass (until
converged) + gradient + ExpSga update, all on the device (irlmx.batch).
``value`` = instance gradient steps per second summed over all GPUs.

Default workload = BASELINE config 3: 128x128 IcyGridWorld, B = 64 instances
per GPU (weak scaling), instance b has p_slip = 0.1 + 0.2*b/B_total, terminal
= last state, identity features, theta0 = 1, demonstrations: 200 synthetic
expert trajectories per instance (irlmx.demos, seed 1234 + b).  Inputs are
resident in HBM before the timed region.

The headline times K steps after W warm-up steps (steady state: the first
step's forward pass runs ~360k sweeps, later ones ~650).  ``first_steps``
reports the run from theta0 = 1 including step 1: steps 1..25 timed one by one
(the warm-up and timed steps are its first W + K; more are run after the timed
region when W + K < 25).

Multi-GPU: one process per GPU (torch.distributed.run); instances are sharded
in contiguous blocks with no collective on the data path.  The process group
is gloo (host-side): it carries only the timing barrier and the max-over-ranks
of the elapsed time, so RCCL is never initialised.

The CPU baseline (rank 0, N = 1) times the reference's own dense numpy
statements (oracle/maxent_oracle.py restates them; maxent.py:98-112, 143-156)
on one instance of the same workload for a bounded sample of sweeps, and
extrapolates with the sweep counts this run logged (mean over instances);
``config1`` times BASELINE config 1 (src/main.py's 5x5 problem: full irl and
irl_causal runs) on the device drop-in and on the oracle, in the same run.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "irl-maxent_amd"))

CONFIGS = {
    # name: (grid size, instances per GPU, description, causal)
    "c3": (128, 64, "BASELINE config 3: 128x128 IcyGridWorld, batch 64 per GPU, fp64", False),
    "c2": (64, 1, "BASELINE config 2 (A=4 pinned variant): 64x64 IcyGridWorld, 1 instance", False),
    "c2s": (64, 1, "BASELINE config 2 (|A|=5): 64x64 IcyGridWorld's four moves + stay, 1 instance, fp64", False),
    "c4": (256, 32, "BASELINE config 4: 256x256 IcyGridWorld, 32 instances per GPU", False),
    "c5": (128, 1, "BASELINE config 5: MaxCausalEnt (soft VI, discount 0.7) on 128x128 IcyGridWorld, "
                   "1 instance per GPU, fp64", True),
}
DISCOUNT = 0.7   # src/main.py's irl_causal discount
FIRST_STEPS = 25

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_FWD = 168                # forward sweep, bytes per state per instance
BYTES_BWD = 152                # backward sweep
BYTES_SOFT = 224               # soft-VI sweep
# fp64 arithmetic per state and sweep: the collapsed
# 5-point stencil is one FMA per point = 10 flop; the forward adds p0 (+1); soft
# VI per action 5 FMAs and the discount product (exp / log not counted)
FLOP_BWD = 10
FLOP_FWD = 11
FLOP_SOFT = 4 * 11
FP64_PEAK_TFS = 78.6           # MI355X FP64 vector (= FP64 matrix) spec peak, MI355X_MICROARCH.md
FP64_LOOP_TFS = 54.8           # tools/diag/dfma_rate.hip mode 0: independent fp64 FMA chains, 2 waves/SIMD


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--size", type=int, default=None, help="override grid size")
    ap.add_argument("--batch", type=int, default=None, help="override instances per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config1", action="store_true", help="skip the config-1 (5x5) same-run timings")
    ap.add_argument("--first-steps", type=int, default=FIRST_STEPS,
                    help="steps from theta0 reported in first_steps (0: off)")
    ap.add_argument("--cpu-sweeps", type=int, default=60, help="timed CPU sweeps per statement")
    fr = ap.add_mutually_exclusive_group()
    fr.add_argument("--full-run", dest="full_run", action="store_true", default=None,
                    help="also run irl to convergence (maxent.py:240-252, eps 1e-4) on a fresh copy of the workload and "
                         "report it under full_run (not part of the headline); default on for config c3 (~11 s), "
                         "off for the others (c4 ~130 s, c5 ~65 s)")
    fr.add_argument("--no-full-run", dest="full_run", action="store_false")
    ap.add_argument("--full-run-eps", type=float, default=1e-4)
    ap.add_argument("--full-run-max-steps", type=int, default=20000, help="cap on gradient steps of the full run")
    ap.add_argument("--no-compact", action="store_true", help="full run without compacting converged instances")
    ap.add_argument("--profile", default=None,
                    help="profiles/<tag>_summary.json of a rocprofv3 run of this workload (default: newest); its "
                         "kernel average and PMC HBM bytes are reported beside the live figures")
    args = ap.parse_args(argv)
    if args.full_run is None:
        args.full_run = args.config == "c3" and not args.size and not args.batch
    return args


def _latest(pattern):
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    return files[-1] if files else None


def _latest_profile(config):
    """The newest profiles/r*_summary.json recorded for this workload config
    (tools/parse_rocprof.py writes the config into it; c3 when absent)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")), reverse=True):
        try:
            if json.load(open(path)).get("config", "c3") == config:
                return path
        except (OSError, ValueError):
            continue
    return None


CPU_DENSE_MAX = 128   # larger dense fp64 tables do not fit host RAM (256x256: 137 GB); extrapolate


def cgroup_cpu_quota():
    """CPUs the cgroup CPU controller grants this process (cpu.max quota / period),
    or None when unlimited or unknown (cgroup v2, then v1)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def usable_cpus():
    """(usable CPUs, affinity CPUs, cgroup quota CPUs or None): the CPUs this
    process may run on (sched_getaffinity) capped by its cgroup CPU quota -- the
    "host cores" BASELINE.md asks the CPU baseline to use, which on a shared GPU
    box is far below os.cpu_count()."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return usable, aff, quota


def blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def cpu_sweep_times(size, p_slip, n_sweeps, causal=False, stay=False):
    """Seconds per sweep of the reference's dense statements on one instance
    (oracle restatement): forward maxent.py:109-112, backward :155-156 (or soft
    VI :329-338), and one call's table copies maxent.py:98-102, 143 (320).

    Above 128x128 the dense table does not fit in host memory: the statements
    are timed at 128x128 and scaled by the dense work ratio (S / 16384)^2.
    ``stay``: config 2's fifth action (P[s, s, 4] = 1) appended to the table."""
    if size > CPU_DENSE_MAX:
        t = cpu_sweep_times(CPU_DENSE_MAX, p_slip, n_sweeps, causal, stay)
        ratio = (size * size / float(CPU_DENSE_MAX * CPU_DENSE_MAX)) ** 2
        t.update(t_f=t["t_f"] * ratio, t_b=t["t_b"] * ratio, t_copy=t["t_copy"] * ratio, ratio=ratio,
                 extrapolated_from=CPU_DENSE_MAX)
        return t
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import maxent_oracle as O
    S = size * size
    t0 = time.perf_counter()
    P = O.icy_gridworld_table(size, p_slip)
    if stay:
        P = np.concatenate([P, np.identity(S)[:, :, None]], axis=2)
    A = P.shape[2]
    t_build = time.perf_counter() - t0
    terminal = [S - 1]
    t0 = time.perf_counter()
    p = np.copy(P)
    p[terminal, :, :] = 0.0
    fw = [np.array(p[:, :, a]) for a in range(A)]
    del p
    bw = [np.array(P[:, :, a]) for a in range(A)]
    t_copy = time.perf_counter() - t0
    del P
    rng = np.random.default_rng(0)
    pi = rng.uniform(0.0, 0.5, (S, A))
    p0 = np.zeros(S)
    p0[0] = 1.0
    d = rng.uniform(0.0, 1.0, S)
    er = np.exp(np.ones(S))
    zs = rng.uniform(0.0, 1.0, S)
    phi = O.terminal_reward(terminal, S)
    r = np.ones(S)

    def fwd_sweep(d):   # maxent.py:109-112
        parts = [fw[a].T.dot(pi[:, a] * d) for a in range(A)]
        nxt = p0 + np.array(parts).sum(axis=0)
        return np.max(np.abs(nxt - d)), nxt

    def bwd_sweep(zs):  # maxent.py:155-156
        za = np.array([er * bw[a].dot(zs) for a in range(A)]).T
        return za.sum(axis=1) * 1e-3

    def soft_sweep(v):  # maxent.py:329-338
        q = np.array([r + DISCOUNT * bw[a].dot(v) for a in range(A)]).T
        nv = phi
        for a in range(A):
            nv = O.softmax2(nv, q[:, a])
        nv = np.array(nv, dtype=float)
        np.max(np.abs(nv - v))
        return nv

    back = soft_sweep if causal else bwd_sweep
    if causal:
        zs = -1e200 * np.ones(S)
    for _ in range(2):
        fwd_sweep(d)
        back(zs)
    t0 = time.perf_counter()
    for _ in range(n_sweeps):
        _, d = fwd_sweep(d)
    t_f = (time.perf_counter() - t0) / n_sweeps
    t0 = time.perf_counter()
    for _ in range(n_sweeps):
        zs = back(zs)
    t_b = (time.perf_counter() - t0) / n_sweeps
    return {"t_f": t_f, "t_b": t_b, "t_copy": t_copy, "t_build": t_build, "n_sweeps": n_sweeps, "size": size,
            "causal": causal, "ratio": 1.0, "extrapolated_from": None, "n_actions": A}


def cpu_sweep_times_all_cores(*args, **kw):
    """cpu_sweep_times with BLAS set to every usable CPU (usable_cpus()); the
    thread count actually in effect is recorded in the result."""
    usable, aff, quota = usable_cpus()
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=usable, user_api="blas")
    except Exception:
        limiter = None
    try:
        t = cpu_sweep_times(*args, **kw)
        t["blas_threads"] = int(blas_threads())
    finally:
        if limiter is not None:
            limiter.restore_original_limits()
    t.update(usable_cpus=usable, affinity_cpus=aff, cgroup_quota_cpus=quota)
    return t


def cpu_baseline_from(t, k_b, k_f):
    """instance-steps/s of the timed statements at this run's mean sweep counts:
    one step = K_b * t_b + K_f * t_f + t_copy."""
    t_step = k_b * t["t_b"] + k_f * t["t_f"] + t["t_copy"]
    S = t["size"] * t["size"]
    sample = (f"dense fp64 {t['size']}x{t['size']} (S={S}, A={t.get('n_actions', 4)}), one instance: {t['n_sweeps']} timed sweeps "
              f"each of maxent.py:109-112 (forward, {t['t_f'] / t['ratio'] * 1e3:.1f} ms) and "
              f"{':329-338 (soft VI' if t['causal'] else ':155-156 (backward'}, "
              f"{t['t_b'] / t['ratio'] * 1e3:.1f} ms) + one call's copies maxent.py:98-102,"
              f"{320 if t['causal'] else 143} ({t['t_copy'] / t['ratio']:.2f} s); step = K_b*t_b + K_f*t_f + "
              f"t_copy with this run's K_b={k_b:.0f}, K_f={k_f:.0f} (means over instances); table build "
              f"{t['t_build']:.1f} s untimed")
    if t["extrapolated_from"]:
        sample = (f"extrapolated: the dense fp64 table does not fit host RAM; per-sweep and copy times "
                  f"measured at {t['extrapolated_from']}x{t['extrapolated_from']} x (S ratio)^2 = "
                  f"{t['ratio']:.0f} -- " + sample)
    out = {"value": 1.0 / t_step, "unit": "instance-steps/s", "cores": int(t.get("blas_threads", blas_threads())),
           "host_cpu_count": os.cpu_count(), "kind": "port", "sample": sample}
    if "usable_cpus" in t:
        out.update(usable_cpus=t["usable_cpus"], affinity_cpus=t["affinity_cpus"],
                   cgroup_quota_cpus=t["cgroup_quota_cpus"],
                   cores_note=("BLAS threads = the CPUs this process may use: sched_getaffinity capped by the "
                               "cgroup CPU quota (host_cpu_count is the whole machine)"))
    return out


def cpu_baseline(size, p_slip, k_b, k_f, n_sweeps, causal=False, stay=False):
    return cpu_baseline_from(cpu_sweep_times_all_cores(size, p_slip, n_sweeps, causal, stay), k_b, k_f)


def config1_timings(device_runs=True):
    """BASELINE config 1 (src/main.py: IcyGridWorld(5, 0.2), 200 demonstrations,
    identity features, ExpSga(linear_decay(0.2)), theta0 = 1): the full irl
    (maxent.py:196-255) and irl_causal (discount 0.7, maxent.py:383-453) runs on
    the device drop-in and on the CPU port (oracle, the reference's numpy
    statements), both timed here.  The 200 demonstrations are the reference's
    own (tests/golden/config1.npz, np.random.seed(0))."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import maxent_oracle as O
    z = np.load(os.path.join(ROOT, "tests", "golden", "config1.npz"))
    P, feats = z["p_transition"], np.identity(25)
    rows = [[tuple(int(v) for v in row) for row in z["traj_flat"][o - n:o]]
            for n, o in zip(z["traj_lens"], np.cumsum(z["traj_lens"]))]
    out = {"workload": "BASELINE config 1: src/main.py 5x5 IcyGridWorld, 200 demos, full runs to eps=1e-4",
           "cpu_cores": int(blas_threads())}
    import maxent as M            # the device drop-in (irl-maxent_amd/maxent.py)
    import trajectory as T        # the drop-in trajectory container (irl-maxent_amd/trajectory.py)
    tjs_dev = [T.Trajectory(r) for r in rows]
    tjs_cpu = [O.Trajectory(r) for r in rows]

    class ExpSga:
        """The caller's optimizer, as src/main.py passes one (optimizer.py:110-167 protocol:
        reset / step, theta *= exp(lr_k * grad) in place, lr_k = 0.2 / (1 + k))."""

        def __init__(self):
            self.k, self.parameters = 0, None

        def reset(self, parameters):
            self.parameters, self.k = parameters, 0

        def step(self, grad, *args, **kwargs):
            lr = 0.2 / (1.0 + self.k)
            self.k += 1
            self.parameters *= np.exp(lr * grad)

    def init(n):                  # optimizer.Constant(1.0)
        return np.ones(n)

    runs = {"irl": lambda m, opt, tjs: m.irl(P, feats, [24], tjs, opt, init),
            "irl_causal": lambda m, opt, tjs: m.irl_causal(P, feats, [24], tjs, opt, init, DISCOUNT)}
    for name, fn in runs.items():
        rec = {}
        if device_runs:
            fn(M, ExpSga(), tjs_dev)                          # warm-up (table upload, kernel load)
            opt = ExpSga()
            t0 = time.perf_counter()
            fn(M, opt, tjs_dev)
            rec["gpu_dropin_s"] = time.perf_counter() - t0
            rec["steps"] = opt.k
            rec["gpu_dropin_steps_per_s"] = opt.k / rec["gpu_dropin_s"]
        opt = O.ExpSga(lr=O.linear_decay(0.2))
        t0 = time.perf_counter()
        _, k = fn(O, opt, tjs_cpu)                           # the oracle's loops return (reward, steps)
        rec["cpu_port_s"] = time.perf_counter() - t0
        rec["cpu_port_steps"] = k
        rec["cpu_port_steps_per_s"] = k / rec["cpu_port_s"]
        if device_runs:
            rec["speedup_vs_cpu"] = rec["cpu_port_s"] / rec["gpu_dropin_s"]
        out[name] = rec
    return out


def stream_copy_gbs(dev, nbytes=1 << 30, reps=5):
    """Device-to-device copy rate (read + write bytes / time) on this GPU: the
    achievable-HBM reference SURVEY.md 8(d) asks for beside the 8 TB/s spec."""
    import torch
    a = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
    c = torch.empty_like(a)
    c.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, c
    torch.cuda.empty_cache()
    return gbs


# ---------------------------------------------------------------------------
# timing core (device-independent: tests drive it with stub steps over gloo)
# ---------------------------------------------------------------------------

def timed_steps(step, steps, warmup, barrier, sync, clock=time.perf_counter):
    """W untimed warm-up steps, then exactly K steps bracketed by barrier + sync
    on both sides.  ``step(i, timed)`` runs step i (0-based from theta0).
    Returns (elapsed seconds of the K timed steps, per-step seconds of all
    W + K steps -- each step ends with a sync, so the per-step clock is exact)."""
    per_step = []
    for i in range(warmup):
        t = clock()
        step(i, False)
        sync()
        per_step.append(clock() - t)
    sync()
    barrier()
    sync()
    t0 = clock()
    for i in range(warmup, warmup + steps):
        t = clock()
        step(i, True)
        sync()
        per_step.append(clock() - t)
    sync()
    barrier()
    sync()
    return clock() - t0, per_step


def headline(elapsed_max, per_gpu, world, steps):
    """(value, ms_per_step): whole-job instance-steps/s over the slowest rank's time."""
    return per_gpu * world * steps / elapsed_max, elapsed_max / steps * 1e3


def kernel_name(mode, plan, width):
    """Symbol of the cluster_kernel instantiation a plan runs (cluster.hip)."""
    return f"void irlmx::cluster_kernel<{mode}, {plan['spt']}, {width}, {plan['layout']}, {plan['threads']}>" \
           f"(irlmx::ClusterArgs)"


def full_run(args, mdp, e_f, p_0, terminal, causal, dev, barrier, world):
    """irl to convergence on this rank's instances (maxent.py:236-255: ``while
    delta > eps``), from theta0 = 1, with converged instances compacted out of
    the batch (irlmx.batch) unless --no-compact.  Returns the record of rank 0
    (wall time = the slowest rank's)."""
    import torch
    from irlmx import ops
    from irlmx.batch import BatchedMaxEnt
    from irlmx.shard import max_over_ranks
    irl = BatchedMaxEnt(mdp, e_f, p_0, terminal, causal=causal, discount=DISCOUNT if causal else None)
    B = irl.batch
    trace = []                       # (step, working batch, seconds, forward sweeps summed over the working set)
    clock = [time.perf_counter()]

    def on_step(m):
        torch.cuda.synchronize()
        now = time.perf_counter()
        trace.append((m.k, int(m.last_forward_sweeps.gt(0).sum()), now - clock[0],
                      float(m.last_forward_sweeps.sum())))
        clock[0] = now
        if m.k % 200 == 0:
            print(f"bench.py full run: step {m.k}, {int(m.active.sum())} of {B} instances active", file=sys.stderr,
                  flush=True)

    ctr0 = ops.counters()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    clock[0] = t0
    _, steps = irl.run(eps=args.full_run_eps, max_steps=args.full_run_max_steps, compact=not args.no_compact,
                       on_step=on_step)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    wall_max = max_over_ranks(wall, dev)
    barrier()
    ctr1 = ops.counters()
    steps = steps.cpu().numpy()
    converged = int((~irl.active).sum())
    work = np.array([w for _, w, _, _ in trace], dtype=np.float64)
    secs = np.array([t for _, _, t, _ in trace])
    changes = [(1, int(work[0]))] + [(int(trace[i][0]), int(work[i])) for i in range(1, len(trace))
                                     if work[i] != work[i - 1]]
    inst_steps = int(steps.sum())
    bw = float(np.mean(irl.last_backward_sweeps.cpu().numpy())) if causal else 2.0 * mdp.n_states
    return {
        "eps": args.full_run_eps, "compact": not args.no_compact, "instances_per_gpu": B,
        "instances_total": B * world, "converged_this_rank": converged,
        "gradient_steps": int(irl.k), "max_steps": args.full_run_max_steps,
        "steps_per_instance": {"min": int(steps.min()), "median": float(np.median(steps)), "max": int(steps.max()),
                               "all": [int(v) for v in steps]},
        "wall_s": wall_max, "instance_steps": inst_steps * world,
        "instance_steps_per_s": inst_steps * world / wall_max,
        "irl_runs_per_s": B * world / wall_max,
        "step1_s": float(secs[0]) if len(secs) else None,
        "seconds_by_working_batch": {str(int(w)): float(secs[work == w].sum()) for w in np.unique(work)},
        "working_batch_changes": changes[:64],
        "forward_sweeps_total": float(sum(f for _, _, _, f in trace)),
        "backward_sweeps_per_instance_step": bw,
        "counters": {k: ctr1[k] - ctr0[k] for k in ctr1},
        "note": ("irl run to max|dtheta| <= eps per instance (maxent.py:240-252) from theta0 = 1 on the bench "
                 "workload; stopped instances are compacted out of the batch before each step (irlmx.batch), "
                 "so only active instances pay sweeps; wall = slowest rank, every step synchronised"),
    }


def rank_device(local_rank, n_devices):
    """The GPU of a rank: one per rank (LOCAL_RANK); more ranks than GPUs (a
    rehearsal of the multi-rank path on a 1-GPU box) share them round-robin."""
    return local_rank % max(1, n_devices)


def main(argv=None):
    args = parse(argv)
    # stdout carries exactly one JSON line: whatever libraries print there (gloo's
    # rendezvous messages under torch.distributed.run) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting {world} GPU(s)", file=sys.stderr)
    if world > 1:
        # host-side group: only the timing barrier and the max-over-ranks travel
        # (no data-path collective) -- RCCL is not needed
        dist.init_process_group(backend="gloo")
    local = rank_device(local, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import irlmx
    irlmx.load()          # prebuilt by __graft_entry__.build(); never compiled per rank
    from irlmx import DeviceMDP, demos, ops
    from irlmx.batch import BatchedMaxEnt

    size, per_gpu, desc, causal = CONFIGS[args.config]
    if (args.size and args.size != size) or (args.batch and args.batch != per_gpu):
        desc += f" [overridden: {args.size or size}x{args.size or size}, {args.batch or per_gpu} instances per GPU]"
    size = args.size or size
    per_gpu = args.batch or per_gpu
    S = size * size
    B_total = per_gpu * world
    from irlmx.shard import instance_slips, max_over_ranks, shard_range
    lo, hi = shard_range(B_total, world, rank)
    ids = np.arange(lo, hi)
    slips = instance_slips(ids, B_total)
    terminal = [S - 1]

    stay = args.config == "c2s"
    mdp = DeviceMDP.icy_gridworld(size, slips, device=dev)
    rv = mdp.row_val.cpu().numpy()       # the four moves: the synthetic expert never stays
    if stay:
        mdp = mdp.with_stay()
    e_f = np.empty((per_gpu, S))
    p_0 = np.empty((per_gpu, S))
    for i, b in enumerate(ids):
        e_f[i], p_0[i], _ = demos.sample(rv[i], size, terminal, 0, n=200, seed=1234 + int(b),
                                         max_len=demos.safety_cap(size))
    irl = BatchedMaxEnt(mdp, e_f, p_0, terminal, causal=causal, discount=DISCOUNT if causal else None)
    plans = {"backward": ops.execution_plan(mdp, "soft_backward" if causal else "backward"),
             "forward": ops.execution_plan(mdp, "forward")}
    # one-time costs (code-object loading of every kernel -- the library's and the
    # torch elementwise kernels of the update --, allocator growth) out of every
    # timed figure: one backward, a 16-sweep forward and an update on the same tables
    prime = BatchedMaxEnt(mdp, e_f, p_0, terminal, causal=causal, discount=DISCOUNT if causal else None)
    svf_p, _, _ = ops.forward_svf(mdp, prime.p_initial, prime.terminal, prime.backward(), max_iter=16)
    prime.update(svf_p)
    prime.last_delta.cpu()
    if args.full_run:   # the full run's stop test, compaction and working-set updates (BatchedMaxEnt.run)
        prime.prime_compaction(args.full_run_eps)
    ops.counters()
    del prime, svf_p
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    stream = torch.cuda.current_stream(dev)
    n_all = args.warmup + args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(max(n_all, args.first_steps))]
    sweeps, bsweeps = [], []

    ctr_steps = []   # library event counters (persistent launches, per-sweep reruns) per step

    def step(i, timed):
        e0, e1, e2 = ev[i]
        c0 = ops.counters() if not timed else None
        e0.record(stream)
        pi = irl.backward()
        e1.record(stream)
        svf, iters, _ = irl.forward(pi)
        e2.record(stream)
        irl.update(svf)
        sweeps.append(iters)
        bsweeps.append(irl.last_backward_sweeps if causal else torch.full_like(iters, 2 * S))
        if c0 is not None:   # (untimed steps only: the counter read is a host call)
            c1 = ops.counters()
            ctr_steps.append((i, {k: c1[k] - c0[k] for k in c0 if c1[k] != c0[k]}))

    ctr_start = ops.counters()
    elapsed, per_step = timed_steps(step, args.steps, args.warmup, barrier, torch.cuda.synchronize)
    elapsed_max = max_over_ranks(elapsed, dev)
    value, ms_per_step = headline(elapsed_max, per_gpu, world, args.steps)

    # steps 1..first_steps from theta0 (after the timed region: never inside it)
    n_first = args.first_steps
    for i in range(n_all, n_first):
        t = time.perf_counter()
        step(i, False)
        torch.cuda.synchronize()
        per_step.append(time.perf_counter() - t)

    ctr_end = ops.counters()
    k_f_all = torch.stack(sweeps).to(torch.float64).cpu().numpy()      # [steps run, B]
    k_b_all = torch.stack(bsweeps).to(torch.float64).cpu().numpy()
    timed = slice(args.warmup, n_all)
    k_f, k_b = k_f_all[timed], k_b_all[timed]
    t_bwd = sum(ev[i][0].elapsed_time(ev[i][1]) for i in range(args.warmup, n_all)) * 1e-3
    t_fwd = sum(ev[i][1].elapsed_time(ev[i][2]) for i in range(args.warmup, n_all)) * 1e-3
    bwd_flop = (FLOP_SOFT if causal else FLOP_BWD) * S * float((k_b - (0 if causal else 1)).sum())
    kern = {"backward": {"bytes": (BYTES_SOFT if causal else BYTES_BWD) * S * float(k_b.sum()), "seconds": t_bwd,
                         "launches": args.steps, "flop": bwd_flop},
            "forward": {"bytes": BYTES_FWD * S * float(k_f.sum()), "seconds": t_fwd, "launches": args.steps,
                        "flop": FLOP_FWD * S * float(k_f.sum())}}
    dom = max(kern, key=lambda k: kern[k]["seconds"])
    kd = kern[dom]
    launch_s = kd["seconds"] / kd["launches"]
    achieved = kd["flop"] / kd["seconds"] / 1e12
    if rank == 0:
        dplan = plans[dom]
        kname = kernel_name(1 if dom == "backward" else 0, dplan, size) if dplan["shape"] == "cluster" else None
        roof = {
            "bound": "fp64-valu", "kernel": kname or f"{dom} pass ({dplan['shape']} shape)",
            "achieved": achieved, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFS,
            "traffic": None,
            "flop_per_launch": kd["flop"] / kd["launches"], "launch_ms": launch_s * 1e3,
            "frac_of_fma_loop": achieved / FP64_LOOP_TFS,
            "note": ("binding resource = the fp64 VALU: every sweep is a chain of fp64 FMAs on registers/LDS "
                     "(10 flop per state for the collapsed 5-point backward stencil, 11 forward, 44 soft VI); "
                     "achieved = algorithmic flop per launch / average launch time (HIP events on the launch "
                     "stream); peak = MI355X FP64 spec; frac_of_fma_loop = vs an independent-FMA loop measured "
                     "on the box (tools/diag/dfma_rate.hip, 54.8 TFLOP/s at the clock fp64 load holds)"),
            # SURVEY 8(d)'s streamed-ELL bytes for the same sweeps, against the PMC-measured HBM bytes:
            # the state and weights stay on chip across sweeps, HBM carries the halo exchanges
            "algorithmic_bytes_per_launch": kd["bytes"] / kd["launches"],
        }
        ppath = args.profile or _latest_profile(args.config)
        default_cfg = not args.size and not args.batch
        if ppath and os.path.exists(ppath) and default_cfg:
            prof = json.load(open(ppath))
            src = os.path.relpath(ppath, ROOT)
            k = prof.get("kernels", {}).get(kname) if kname else None
            if k and prof.get("config", "c3") == args.config:
                roof["rocprof_avg_ms"] = k["avg_ms"]
                roof["frac_rocprof"] = kd["flop"] / kd["launches"] / (k["avg_ms"] * 1e-3) / 1e12 / FP64_PEAK_TFS
                roof["rocprof_source"] = f"{src}: rocprofv3 --kernel-trace --stats average of {kname}"
            tr = prof.get("traffic", {}).get(dom)
            if tr and tr.get("kernel") == kname and prof.get("config", "c3") == args.config:
                roof["traffic"] = tr["hbm_bytes_per_launch"]
                roof["traffic_source"] = (f"{src}: FETCH_SIZE + WRITE_SIZE (KiB x 1024) of one {dom} dispatch, "
                                          f"separate --pmc passes")
                roof["hbm_frac"] = tr["hbm_bytes_per_launch"] / launch_s / 1e9 / HBM_PEAK_GBS
                roof["onchip_reuse_factor"] = roof["algorithmic_bytes_per_launch"] / tr["hbm_bytes_per_launch"]
        out = {
            "metric": "IRL gradient steps/sec (VI + SVF sweep), NxN grid batch B",
            "value": value,
            "unit": "instance-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device-built IcyGridWorld tables, seeded synthetic expert demos)",
            "config": {"workload": desc, "grid": f"{size}x{size}", "n_states": S, "n_actions": mdp.n_actions,
                       "batch_per_gpu": per_gpu, "global_batch": B_total, "eps_svf": 1e-5,
                       "parallelism": f"instances sharded over {world} GPU(s), no collective"},
            "plans": plans,
            "sweeps": {"backward_per_step": float(k_b.mean()), "forward_mean": float(k_f.mean()),
                       "forward_max": float(k_f.max())},
            "phase_s": {"backward": t_bwd, "forward": t_fwd},
            "roofline": roof,
            "per_kernel": {k: {"ms_per_launch": v["seconds"] / v["launches"] * 1e3,
                               "achieved_TFLOPs": v["flop"] / v["seconds"] / 1e12,
                               "algorithmic_GBs": v["bytes"] / v["seconds"] / 1e9}
                           for k, v in kern.items()},
        }
        if n_first:
            t_first = sum(per_step[:n_first])
            bwd_ms = [ev[i][0].elapsed_time(ev[i][1]) for i in range(n_first)]
            fwd_ms = [ev[i][1].elapsed_time(ev[i][2]) for i in range(n_first)]
            out["first_steps"] = {
                "steps": n_first, "seconds": t_first, "instance_steps_per_s": per_gpu * n_first / t_first,
                "step1_ms": per_step[0] * 1e3,
                # step 1's phases (HIP events on the launch stream): backward, forward to convergence
                # from the unit reward, and the rest (gradient, update, host work) = step1_ms - both
                "step1_backward_ms": bwd_ms[0], "step1_forward_ms": fwd_ms[0],
                "step1_other_ms": per_step[0] * 1e3 - bwd_ms[0] - fwd_ms[0],
                "step1_forward_us_per_sweep": fwd_ms[0] * 1e3 / max(1.0, float(k_f_all[0].max())),
                "backward_ms": [round(v, 3) for v in bwd_ms], "forward_ms": [round(v, 3) for v in fwd_ms],
                # per untimed step: library events that occurred (persistent launches, per-sweep reruns
                # after a non-finite value, a failed co-residency rendezvous or an exchange timeout)
                "events": {str(i + 1): c for i, c in ctr_steps if i < n_first},
                "forward_sweeps_mean": [float(v) for v in k_f_all[:n_first].mean(axis=1)],
                "note": ("steps 1..N of irl from theta0 = 1 on this GPU's instances, each timed to its own sync "
                         "(the warm-up and timed steps are the first W + K); step 1's forward runs to convergence "
                         "from the unit reward (~360k sweeps at 128x128)")}
        out["counters"] = {k: ctr_end[k] - ctr_start[k] for k in ctr_end}
        out["roofline"]["stream_copy_GBs"] = stream_copy_gbs(dev)
        if world == 1 and not args.no_cpu_baseline:
            t = cpu_sweep_times_all_cores(size, float(slips[0]), args.cpu_sweeps, causal, stay)
            out["cpu_baseline"] = cpu_baseline_from(t, float(k_b.mean()), float(k_f.mean()))
            out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            if n_first:
                kb_first = k_b_all[:n_first].mean(axis=1)
                kf_first = k_f_all[:n_first].mean(axis=1)
                t_cpu = float(np.sum(kb_first * t["t_b"] + kf_first * t["t_f"] + t["t_copy"]))
                out["first_steps"]["cpu_baseline_instance_steps_per_s"] = n_first / t_cpu
                out["first_steps"]["speedup_vs_cpu"] = out["first_steps"]["instance_steps_per_s"] * t_cpu / n_first
            if not args.no_config1:
                out["config1"] = config1_timings()
    if args.full_run:
        fr = full_run(args, mdp, e_f, p_0, terminal, causal, dev, barrier, world)
        if rank == 0:
            if "cpu_baseline" in out:
                # the reference's statements for the same run: every instance-step pays K_b backward
                # sweeps and one call's copies, plus the forward sweeps it logged
                t_cpu = fr["instance_steps"] * (fr["backward_sweeps_per_instance_step"] * t["t_b"] + t["t_copy"]) \
                    + fr["forward_sweeps_total"] * t["t_f"]
                fr["cpu_baseline_s"] = t_cpu
                fr["speedup_vs_cpu"] = t_cpu / fr["wall_s"]
            out["full_run"] = fr
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
