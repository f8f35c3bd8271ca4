"""Benchmark: env-steps/s of the drop-in Env.step on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
the driver launches one rank per GPU with torch.distributed.run. Rank 0
prints ONE JSON line.

Workload (BASELINE.json configs[2]): per GPU 65,536 envs x
3 agents x 3 obstacles, fp32, default reward factors, episode_len 200, native
(Philox) re-init. Actions: 64 pre-generated device tensors, angle ~
U(-0.5, 0.5) rad, acceleration ~ U(-0.5, 0.5), cycled. Each rank owns an
independent slice of global env ids [rank*P, (rank+1)*P) (weak scaling); the
data path has no collective. A step = one ``Env.step`` call, through the
Python API, returning fresh observation/reward/done tensors.

Timing: W untimed steps; barrier + synchronize; K timed steps; synchronize +
barrier; the max over ranks. value = N*P*K / max time.

roofline: the step kernel's average duration from HIP events recorded on the
launch stream (torch's current stream, where Env.step enqueues) around the
timed region, divided by K (an upper bound: inter-kernel gaps are included),
against the algorithmic bytes per env-step (read 28A+8O+13, write
20A+4A*D+11: 336 B at A3/O3) and the 8 TB/s HBM peak. kernel_us_graph: the
same from replays of a hipGraph of back-to-back Env.step launches, for
reference. traffic: HBM bytes per launch from the committed rocprofv3 PMC
summary for this config (profiles/), or null.

cpu_baseline (rank 0, N=1): oracle/torch_ref.py - the reference's step
restated with its own execution structure in eager PyTorch on the host CPU -
timed on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0


def alg_bytes_per_env(A, O):
    D = 2 + 2 * O + 2 * (A - 1)
    return (28 * A + 8 * O + 13) + (20 * A + 4 * A * D + 11)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--agents", type=int, default=3)
    ap.add_argument("--obstacles", type=int, default=3)
    ap.add_argument("--cpu-baseline", choices=("auto", "on", "off"), default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_summary.json"))
    return ap.parse_args()


def make_env(pkg, P, A, O, device, rank):
    args = pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O)
    params = pkg.set_env_params(args, device)
    params["rng"] = "native"
    params["seed"] = 20251003
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


def kernel_time_us(env, actions, n=25, replays=12):
    """Average step-kernel time from HIP events on the launch stream around
    replays of a hipGraph holding n back-to-back Env.step launches (no host
    gaps between kernels; each interval includes the graph's inter-kernel
    boundary, so this slightly overstates the kernel duration)."""
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
    graph.replay()
    torch.cuda.synchronize()
    per = []
    for _ in range(replays):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        graph.replay()
        e.record()
        e.synchronize()
        per.append(s.elapsed_time(e) * 1e3 / n)
    per.sort()
    return sum(per) / len(per), per[len(per) // 2]


def cpu_baseline(P, A, O, seconds, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from torch_ref import TorchRefEnv
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        env = TorchRefEnv(P, A, O, seed=7)
        g = torch.Generator().manual_seed(99)
        acts = [torch.stack([torch.rand(P, A, generator=g) - 0.5,
                             torch.rand(P, A, generator=g) - 0.5], 2) for _ in range(4)]
        env.step(acts[0])
        t0 = time.perf_counter()
        n = 0
        while True:
            env.step(acts[n % 4])
            n += 1
            if time.perf_counter() - t0 > seconds or n >= 1000:
                break
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return P * n / dt, n, dt


def load_traffic(path, workload):
    try:
        with open(path) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return None
    ent = pmc.get(workload)
    if not ent:
        return None
    return ent.get("hbm_bytes_per_launch")


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world > 1:
            raise SystemExit(f"WORLD_SIZE={world} but --gpus {a.gpus}")
    # MARLNAV_BENCH_BACKEND=gloo rehearses the N>1 path on fewer GPUs than
    # ranks (ranks share devices; reductions on the host)
    backend = os.environ.get("MARLNAV_BENCH_BACKEND", "nccl")
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
    P, A, O = a.envs, a.agents, a.obstacles
    env = make_env(pkg, P, A, O, device, rank)
    actions = make_actions(P, A, device, rank)

    for i in range(a.warmup):
        env.step(actions[i % len(actions)])

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(a.steps):
        env.step(actions[i % len(actions)])
    ev1.record()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    dt = pkg.shard.max_over_ranks(dt, red_dev)
    kern_avg = ev0.elapsed_time(ev1) * 1e3 / a.steps  # us per step-kernel, timed region

    kern_graph, kern_med = kernel_time_us(env, actions)
    per_env = alg_bytes_per_env(A, O)
    launch_bytes = per_env * P
    achieved = launch_bytes / (kern_avg * 1e-6) / 1e9
    workload = f"P{P}_A{A}_O{O}"
    traffic = load_traffic(a.pmc, workload)

    cpu = None
    want_cpu = a.cpu_baseline == "on" or (a.cpu_baseline == "auto" and world == 1)
    if rank == 0 and want_cpu:
        threads = a.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        v, n, secs = cpu_baseline(P, A, O, a.cpu_seconds, threads)
        cpu = {"value": v, "unit": "env-steps/s", "cores": threads, "kind": "port",
               "sample": (f"oracle/torch_ref.py (reference step structure, eager torch "
                          f"CPU): {n} steps x {P} envs x {A} agents x {O} obstacles "
                          f"in {secs:.1f} s after 1 warm-up step; host os.cpu_count()="
                          f"{os.cpu_count()}")}

    counters = pkg.shard.sum_over_ranks([env._num_trunc, env._num_col, env._num_tar], red_dev)
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: native triangle init, U(-0.5,0.5) angle/accel actions",
            "config": {"workload": f"{P} envs x {A} agents x {O} obstacles per GPU "
                                   f"(BASELINE configs[2]); Env.step via C ABI",
                       "envs_per_gpu": P, "agents": A, "obstacles": O,
                       "global_envs": world * P, "episode_len": 200,
                       "parallelism": f"independent env slices x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel_us_avg": kern_avg, "kernel_us_graph": kern_graph,
                         "kernel_us_graph_median": kern_med,
                         "alg_bytes_per_launch": launch_bytes,
                         "alg_bytes_per_env_step": per_env},
            "cpu_baseline": cpu,
            "episode_counters": counters,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
