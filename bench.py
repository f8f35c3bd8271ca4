"""Benchmark: env-steps/s of the drop-in Env.step on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
the driver launches one rank per GPU with torch.distributed.run. Run as a
plain process with ``--gpus N`` > 1, bench.py starts that launcher itself
(before touching the GPU) and exits with its status. Rank 0 prints ONE JSON
line.

Workload (BASELINE.json configs[2]): per GPU 65,536 envs x
3 agents x 3 obstacles, fp32, default reward factors, episode_len 200, native
(Philox) re-init. Actions: 64 pre-generated device tensors, angle ~
U(-0.5, 0.5) rad, acceleration ~ U(-0.5, 0.5), cycled. Each rank owns an
independent slice of global env ids [rank*P, (rank+1)*P) (weak scaling); the
data path has no collective. A step = one ``Env.step`` call, through the
Python API, returning fresh observation/reward/done tensors.

Timing: a GPU clock ramp (``--prewarm`` seconds of back-to-back steps of a
second, scratch Env of the same shape, before anything of the timed Env
runs: an idle MI355X starts the first milliseconds of a process at low
clocks, which at the driver's 20-step setting was the difference between
9 and 22 us per step on the same box); W untimed steps of the timed Env;
barrier + synchronize; K timed steps; synchronize + barrier; the max over
ranks. value = N*P*K / max time.

roofline (the step kernel): ``launch_us`` = the step kernel's average launch
duration by HIP events on the launch stream (``event_launch_us``): further
passes of the same K Env.step calls right after the timed region, each behind
a short device spin so that the events bracket the K launches back to back
(the timed pass itself carries no events: recording one there adds ~13 us of
GPU-side marker processing per region, scripts/diag/sync_overhead.py); the
median of three. ``achieved`` = algorithmic bytes per launch (read
28A+8O+13, write 20A+4A*D+11 per env-step: 336 B at A3/O3) / ``launch_us``,
against the 8 TB/s HBM peak; it agrees with a rocprofv3 average of the same
launches (profiles/). Beside it: ``timed_region_frac``, the same bytes over
``ms_per_step`` (the timed region's fixed first-launch and closing
synchronisation cost included: a lower bound). Cross-check: ``graph_replay_launch_us``, the
same launches back to back from a hipGraph of a second Env of the same shape
(the timed env's state and counters untouched), which is what a rocprofv3
kernel duration of back-to-back launches measures. ``traffic``: HBM bytes per
launch from the committed rocprofv3 PMC summary for this config (profiles/;
not measured in this run - the source is named), or null.

cpu_baseline (rank 0 of an N=1 run, after the timed region; null at N>1 unless
--cpu-baseline on): oracle/torch_ref.py - the reference's step
restated with its own execution structure in eager PyTorch (pinned bit for
bit to the reference's golden vectors, tests/test_torch_ref.py) - timed on
the host CPU with all available cores and with one thread on a bounded
sample of the same workload; plus the same restatement run eagerly on the
GPU (how the reference itself runs there).
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch does not initialise the GPU)

HBM_PEAK_GBS = 8000.0
SPIN_CYCLES = 200_000  # ~0.1 ms of device spin (bench main: the event pass)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")


def alg_bytes_per_env(A, O):
    D = 2 + 2 * O + 2 * (A - 1)
    return (28 * A + 8 * O + 13) + (20 * A + 4 * A * D + 11)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", type=int, choices=(0, 1, 2, 3, 4), default=None,
                    help="a BASELINE.json configs[i] shape (overrides --envs/--agents/"
                         "--obstacles); 4 = 131072 envs split over the --gpus ranks")
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--agents", type=int, default=3)
    ap.add_argument("--obstacles", type=int, default=3)
    ap.add_argument("--cpu-baseline", choices=("auto", "on", "off"), default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="seconds of CPU-baseline work per thread setting")
    ap.add_argument("--pmc", default=PMC_SUMMARY)
    ap.add_argument("--prewarm", type=float, default=0.3,
                    help="seconds of scratch-Env steps before the timed Env starts")
    return ap.parse_args(argv)


# BASELINE.json configs: (envs, agents, obstacles); configs[4]'s envs are the
# global count, split over the ranks (strong scaling)
BASELINE_CONFIGS = {0: (2, 3, 3), 1: (1024, 3, 8), 2: (65536, 3, 3), 3: (4096, 16, 32),
                    4: (131072, 3, 3)}


def workload(a, world):
    """(envs per GPU, A, O, label, scaling) of this run."""
    if a.config is not None:
        P, A, O = BASELINE_CONFIGS[a.config]
        if a.config == 4:
            if P % world:
                raise SystemExit(f"configs[4]: 131072 envs do not split over {world} ranks")
            return (P // world, A, O,
                    f"BASELINE configs[4]: 131072 envs x 3 agents x 3 obstacles over {world} "
                    f"GPU(s), {P // world} per GPU", "strong")
        return P, A, O, f"BASELINE configs[{a.config}]", "weak"
    P, A, O = a.envs, a.agents, a.obstacles
    for i, shape in BASELINE_CONFIGS.items():
        if (P, A, O) == shape and i != 4:
            return P, A, O, f"BASELINE configs[{i}]", "weak"
    if (P * world, A, O) == BASELINE_CONFIGS[4]:
        return P, A, O, (f"BASELINE configs[4]: 131072 envs x 3 agents x 3 obstacles over "
                         f"{world} GPU(s), {P} per GPU"), "weak"
    return P, A, O, "custom", "weak"


def self_launch(a):
    """--gpus N > 1 outside torch.distributed.run: start the launcher as a
    child (this process has not touched the GPU) and return its status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def make_env(pkg, P, A, O, device, rank, seed=20251003):
    args = pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O)
    params = pkg.set_env_params(args, device)
    params["rng"] = "native"
    params["seed"] = seed
    params["env_offset"], _ = pkg.shard.weak_slice(rank, P)
    return pkg.Env(params)


def make_actions(P, A, device, rank, n=64):
    g = torch.Generator(device=device)
    g.manual_seed(1234 + rank)
    out = []
    for _ in range(n):
        th = torch.rand(P, A, generator=g, device=device) - 0.5
        acc = torch.rand(P, A, generator=g, device=device) - 0.5
        out.append(torch.stack([th, acc], 2).contiguous())
    return out


def kernel_time_us(env, actions, n=25, replays=12, per_event=8):
    """Average step-launch duration: HIP events on the launch stream around
    ``per_event`` back-to-back replays of a hipGraph holding n Env.step
    launches of ``env`` (each interval includes the graph's inter-kernel
    boundary, as a back-to-back rocprofv3 kernel duration does; the ~13 us an
    event pair adds on the GPU is spread over n * per_event launches).
    ``replays`` such measurements; returns (mean, median) in us per launch."""
    env.allow_graph_capture = True  # replays repeat the captured re-init draws: timing only
    graph = capture_steps(env, actions, n)
    graph.replay()
    torch.cuda.synchronize()
    per = []
    for _ in range(replays):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(per_event):
            graph.replay()
        e.record()
        e.synchronize()
        per.append(s.elapsed_time(e) * 1e3 / (n * per_event))
    per.sort()
    return sum(per) / len(per), per[len(per) // 2]


def capture_steps(env, actions, n):
    """A hipGraph of n back-to-back Env.step launches of ``env`` (which must
    allow graph capture; replays repeat the captured re-init draws)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for i in range(3):
            env.step(actions[i % len(actions)])
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for i in range(n):
            env.step(actions[i % len(actions)])
    return graph


def prewarm(env, actions, seconds):
    """GPU clock ramp: back-to-back steps of a scratch Env for ``seconds``
    (nothing of the timed Env runs here), as replays of a hipGraph of 64
    steps, so the GPU stays busy without host gaps (under rocprofv3, whose
    per-launch host overhead exceeds a step, host-launched steps would run
    isolated). Returns the steps taken."""
    env.allow_graph_capture = True  # scratch Env: the replays' repeated draws are irrelevant
    graph = capture_steps(env, actions, 64)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            graph.replay()
            n += 64
        torch.cuda.synchronize()
    env.allow_graph_capture = False
    return n


def host_cpu_facts():
    model = platform.processor() or "?"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return {"model": model, "os_cpu_count": os.cpu_count(),
            "sched_getaffinity": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def time_torch_ref(P, A, O, seconds, threads=None, device="cpu"):
    """Steps/s of oracle/torch_ref.py over a bounded sample; returns
    (env-steps/s, steps, seconds)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from torch_ref import TorchRefEnv
    prev = torch.get_num_threads()
    if threads:
        torch.set_num_threads(threads)
    try:
        env = TorchRefEnv(P, A, O, seed=7, device=device)
        g = torch.Generator().manual_seed(99)
        acts = [torch.stack([torch.rand(P, A, generator=g) - 0.5,
                             torch.rand(P, A, generator=g) - 0.5], 2).to(device)
                for _ in range(4)]
        env.step(acts[0])
        if device != "cpu":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        while True:
            env.step(acts[n % 4])
            n += 1
            if time.perf_counter() - t0 > seconds or n >= 2000:
                break
        if device != "cpu":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return P * n / dt, n, dt


def cpu_baseline(P, A, O, seconds, device):
    facts = host_cpu_facts()
    # all cores the process may run on (the cgroup quota caps how many of
    # them it gets; more threads than that only oversubscribe)
    n_all = facts["sched_getaffinity"]
    if facts["cgroup_cpu_quota"]:
        n_all = max(1, min(n_all, int(facts["cgroup_cpu_quota"])))
    v_all, n1, s1 = time_torch_ref(P, A, O, seconds, threads=n_all)
    v_one, n2, s2 = time_torch_ref(P, A, O, seconds, threads=1)
    v_gpu, n3, s3 = time_torch_ref(P, A, O, seconds / 2, device=str(device))
    return {"value": v_all, "unit": "env-steps/s", "cores": n_all, "kind": "port",
            "value_1thread": v_one,
            "sample": (f"oracle/torch_ref.py (the reference's step structure, eager torch; "
                       f"bit-exact vs the reference goldens): {P} envs x {A} agents x {O} "
                       f"obstacles, {n1} steps in {s1:.1f} s on {n_all} threads, {n2} steps "
                       f"in {s2:.1f} s on 1 thread, after 1 warm-up step"),
            "host": facts,
            "secondary_eager_torch_gpu": {"value": v_gpu, "unit": "env-steps/s",
                                          "sample": f"same restatement on {device}: {n3} "
                                                    f"steps in {s3:.1f} s"}}


def load_traffic(path, workload):
    try:
        with open(path) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return None, None
    ent = pmc.get(workload)
    if not ent:
        return None, None
    return ent.get("hbm_bytes_per_launch"), ent.get("source", os.path.relpath(path, ROOT))


def default_backend():
    """torch.distributed backend of the N>1 harness: gloo unless
    MARLNAV_BENCH_BACKEND says otherwise."""
    b = os.environ.get("MARLNAV_BENCH_BACKEND", "gloo")
    if b not in ("gloo", "nccl"):
        raise SystemExit(f"MARLNAV_BENCH_BACKEND={b!r}: gloo or nccl")
    return b


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and a.gpus > 1 and "LOCAL_RANK" not in os.environ:
        return self_launch(a)
    if world != a.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {a.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # The N>1 harness (barriers, the max-over-ranks time, summed counters,
    # the gathered slice table) runs over gloo on the host by default: the
    # data path has no collective, so no RCCL is needed.
    # MARLNAV_BENCH_BACKEND=nccl opts into RCCL. Under gloo, ranks beyond the
    # visible GPUs share them (a rehearsal of N ranks on fewer GPUs).
    backend = default_backend()
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    red_dev = device if backend == "nccl" else None

    import marlnav_amd as pkg
    P, A, O, cfg_name, scaling = workload(a, world)
    env = make_env(pkg, P, A, O, device, rank)
    actions = make_actions(P, A, device, rank)
    kenv = make_env(pkg, P, A, O, device, rank, seed=20251004)
    prewarm_steps = prewarm(kenv, actions, a.prewarm)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()   # the first timing event of a process is slow to record:
    ev1.record()   # pay that here, outside the timed region
    ev1.synchronize()

    for i in range(a.warmup):
        env.step(actions[i % len(actions)])

    def barrier():
        if dist is not None:
            dist.barrier()

    # the timed region: exactly K steps between barrier + synchronize pairs,
    # with no instrumentation inside (a timing-event record in the region
    # costs ~13 us of GPU marker processing per region at 65536 envs:
    # scripts/diag/sync_overhead.py, profiles/r02_sync_overhead.txt)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        env.step(actions[i % len(actions)])
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    dt = pkg.shard.max_over_ranks(dt, red_dev)
    counters = pkg.shard.sum_over_ranks([env._num_trunc, env._num_col, env._num_tar], red_dev)
    slices = pkg.shard.gather_slices(env._env_offset, P)

    # the same K steps again with HIP events on the launch stream around
    # them: the GPU-side time per step of the timed loop (diagnostic; not
    # the value)
    # A short device spin ahead of the start event keeps the queue busy while
    # the host enqueues the first steps, so the region holds the K launches
    # back to back and not the host's start-up gap before the first one
    # (at K = 20 that gap moved launch_us by up to 1.5 us between runs on one
    # box); three such passes, the median.
    barrier()
    torch.cuda.synchronize()
    regions = []
    for rep in range(3):
        torch.cuda._sleep(SPIN_CYCLES)
        ev0.record()
        for i in range(a.steps):
            env.step(actions[((2 + rep) * a.steps + i) % len(actions)])
        ev1.record()
        torch.cuda.synchronize()
        regions.append(ev0.elapsed_time(ev1) * 1e3 / a.steps)
    region_us = sorted(regions)[1]

    kern_us, kern_med = kernel_time_us(kenv, actions)
    del kenv
    per_env = alg_bytes_per_env(A, O)
    launch_bytes = per_env * P
    # roofline.achieved: algorithmic bytes per launch over the event-timed
    # average launch duration (above, which agrees with a rocprofv3 average of
    # the same launches); timed_region_frac: over the timed region's time per
    # step (one launch per step, the region's fixed synchronisation cost
    # included: a lower bound on the kernel's own rate). The graph-replay
    # figure is kept beside them.
    step_us = dt * 1e6 / a.steps
    achieved = launch_bytes / (region_us * 1e-6) / 1e9
    timed_frac = launch_bytes / (step_us * 1e-6) / 1e9 / HBM_PEAK_GBS
    traffic, traffic_src = load_traffic(a.pmc, f"P{P}_A{A}_O{O}")

    cpu = None
    # (the CPU baseline belongs to the N=1 line; --cpu-baseline on forces it)
    want_cpu = a.cpu_baseline == "on" or (a.cpu_baseline == "auto" and world == 1)
    if rank == 0 and want_cpu:
        cpu = cpu_baseline(P, A, O, a.cpu_seconds, device)

    if rank == 0:
        line = {
            "metric": "env-steps/sec (whole node) at 3 agents; 1/2/4/8-GPU scaling + %HBM roofline",
            "value": world * P * a.steps / dt,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: native triangle init, U(-0.5,0.5) angle/accel actions",
            "config": {"workload": f"{P} envs x {A} agents x {O} obstacles per GPU "
                                   f"({cfg_name}); Env.step via C ABI",
                       "baseline_config": cfg_name,
                       "envs_per_gpu": P, "agents": A, "obstacles": O,
                       "global_envs": world * P, "episode_len": 200,
                       "parallelism": f"independent env slices x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "launch_us": region_us,
                         "launch_us_source": "HIP events on the launch stream, K back-to-back "
                                             "Env.step launches after the timed region (median of 3)",
                         "timed_region_frac": timed_frac,
                         "timed_region_launch_us": step_us,
                         "event_launch_us": region_us,
                         "event_launch_us_passes": regions,
                         "graph_replay_launch_us": kern_us,
                         "graph_replay_launch_us_median": kern_med,
                         "alg_bytes_per_launch": launch_bytes,
                         "alg_bytes_per_env_step": per_env},
            "cpu_baseline": cpu,
            **({} if cpu is not None else
               {"cpu_baseline_note": "off" if a.cpu_baseline == "off"
                else "measured on rank 0 of the N=1 run only"}),
            "prewarm": {"seconds": a.prewarm, "scratch_env_steps": prewarm_steps},
            "episode_counters": counters,
            "ranks": [{"rank": r, "env_offset": off, "envs": n} for r, off, n in slices],
            "dist_backend": backend if world > 1 else None,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
