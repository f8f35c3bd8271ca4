"""The N>1 path on CPU with gloo, world size 2: shard layout, sharding
invariance of the native re-init stream (keyed on global env ids) through
the oracle, and the harness reductions bench.py uses."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import marlnav_amd as pkg
    import oracle as orc
    from marlnav_amd.environment import make_cparams
    off, n = pkg.shard.strong_slice(total, rank, world)
    init = pkg.init_sampler(dict(pkg.set_init_params(
        pkg.default_args(num_parallel=n, num_obstacles=3), "cpu"), num_agents=3))
    pr = make_cparams({"min_speed": 3., "max_speed": 10., "min_accel": -.5, "max_accel": .5,
                       "_risk_factor": 0., "_distance_factor": 0., "_heading_factor": 500.,
                       "_target_factor": 500., "_soft_factor": 500., "_bond_factor": 10.,
                       "episode_len": 6}, init=init, seed=4242)
    form = np.concatenate([init.formation.numpy().ravel(), init.target_point.numpy()])
    dm = orc.make_dims(n, 3, 3, env_offset=off)
    st, ob, tg = orc.reinit_all(dm, pr, form, 0)
    sn, te = np.zeros(n, np.float32), np.zeros(n, np.bool_)
    g = np.random.default_rng(11)
    acts_all = g.uniform(-0.5, 0.5, size=(20, total, 3, 2)).astype(np.float32)
    cnt = np.zeros(3, np.int64)
    for k in range(20):
        o = orc.step(dm, pr, st, ob, tg, sn, te, acts_all[k, off:off + n], formation=form,
                     step_idx=k + 1)
        st, ob, tg, sn, te = (o[x] for x in ("states", "obstacles", "target", "step_num",
                                             "terminates"))
        cnt += o["counters"]
    gathered = [None] * world
    dist.all_gather_object(gathered, (off, st, ob))
    tmax = pkg.shard.max_over_ranks(1.0 + rank)
    csum = pkg.shard.sum_over_ranks(cnt.tolist())
    slices = pkg.shard.gather_slices(off, n)   # rank 0's check: every rank, no gaps
    if rank == 0:
        np.savez(os.path.join(out_dir, "dist.npz"),
                 st=np.concatenate([x[1] for x in sorted(gathered, key=lambda t: t[0])]),
                 ob=np.concatenate([x[2] for x in sorted(gathered, key=lambda t: t[0])]),
                 tmax=tmax, csum=np.asarray(csum), slices=np.asarray(slices))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_one_batch(tmp_path, pkg):
    import oracle as orc
    from marlnav_amd.environment import make_cparams
    total, world = 301, 2
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world,
             join=True)
    res = np.load(tmp_path / "dist.npz")
    assert float(res["tmax"]) == 2.0
    np.testing.assert_array_equal(res["slices"], [[0, 0, 151], [1, 151, 150]])
    # single-process reference over the whole batch
    init = pkg.init_sampler(dict(pkg.set_init_params(
        pkg.default_args(num_parallel=total, num_obstacles=3), "cpu"), num_agents=3))
    pr = make_cparams({"min_speed": 3., "max_speed": 10., "min_accel": -.5, "max_accel": .5,
                       "_risk_factor": 0., "_distance_factor": 0., "_heading_factor": 500.,
                       "_target_factor": 500., "_soft_factor": 500., "_bond_factor": 10.,
                       "episode_len": 6}, init=init, seed=4242)
    form = np.concatenate([init.formation.numpy().ravel(), init.target_point.numpy()])
    dm = orc.make_dims(total, 3, 3)
    st, ob, tg = orc.reinit_all(dm, pr, form, 0)
    sn, te = np.zeros(total, np.float32), np.zeros(total, np.bool_)
    acts_all = np.random.default_rng(11).uniform(-0.5, 0.5, size=(20, total, 3, 2)).astype(
        np.float32)
    cnt = np.zeros(3, np.int64)
    for k in range(20):
        o = orc.step(dm, pr, st, ob, tg, sn, te, acts_all[k], formation=form, step_idx=k + 1)
        st, ob, tg, sn, te = (o[x] for x in ("states", "obstacles", "target", "step_num",
                                             "terminates"))
        cnt += o["counters"]
    np.testing.assert_array_equal(res["st"], st)
    np.testing.assert_array_equal(res["ob"], ob)
    np.testing.assert_array_equal(res["csum"], cnt)
    assert cnt[0] > 0  # truncations happened, so re-inits were drawn per shard


@pytest.mark.parametrize("total,world", [(10, 3), (65536, 8), (7, 8), (131072, 8)])
def test_strong_slices_partition(pkg, total, world):
    got = [pkg.shard.strong_slice(total, r, world) for r in range(world)]
    assert sum(n for _, n in got) == total
    assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(world - 1))
    assert max(n for _, n in got) - min(n for _, n in got) <= 1
    assert pkg.shard.weak_slice(3, 65536) == (3 * 65536, 65536)


def test_bench_self_launches_n_ranks(monkeypatch):
    """`python bench.py --gpus N` outside torch.distributed.run starts the
    launcher with N ranks on 127.0.0.1 (before any GPU call) and returns its
    status; it never times one GPU and reports n_gpus 1 for --gpus N."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    for k in ("WORLD_SIZE", "LOCAL_RANK", "RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "20", "--warmup", "5"])
    assert bench.main() == 7
    (cmd,) = calls
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == ["--gpus", "4", "--steps", "20", "--warmup", "5"]
    # under the launcher, a rank count that disagrees with --gpus is an error
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_RANK", "0")
    with pytest.raises(SystemExit):
        bench.main()


def _gap_worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import marlnav_amd as pkg
    try:
        pkg.shard.gather_slices(rank * 100 + (7 if rank == 1 else 0), 100)
        msg = "no error"
    except RuntimeError as e:
        msg = str(e)
    with open(os.path.join(out_dir, f"gap{rank}.txt"), "w") as fh:
        fh.write(msg)
    dist.destroy_process_group()


def test_gather_slices_rejects_a_gap(tmp_path):
    """A rank whose slice does not start where the previous one ends fails
    the gathered-slice check on every rank (bench.py's rank-0 table)."""
    mp.spawn(_gap_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert "rank 1 owns envs from 107, expected 100" in (tmp_path / f"gap{r}.txt").read_text()


def test_bench_default_backend_is_gloo(monkeypatch):
    """The N>1 harness defaults to gloo (host-side reductions, no RCCL);
    nccl only on request; anything else is refused."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    monkeypatch.delenv("MARLNAV_BENCH_BACKEND", raising=False)
    assert bench.default_backend() == "gloo"
    monkeypatch.setenv("MARLNAV_BENCH_BACKEND", "nccl")
    assert bench.default_backend() == "nccl"
    monkeypatch.setenv("MARLNAV_BENCH_BACKEND", "mpi")
    with pytest.raises(SystemExit):
        bench.default_backend()
