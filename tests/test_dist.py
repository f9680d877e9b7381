"""CPU: the multi-GPU path (instance sharding, per-rank inputs, stats all_gather,
max-over-ranks timing) with world_size = 2 on the gloo backend.

The per-rank solver here is the C++ CPU oracle (the GPU is exercised by the
gpu tests and by bench.py); what is tested is that a sharded run reproduces the
single-process run instance-for-instance and that the collectives assemble it.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _closed_loop_shard(P, steps, N):
    from oracle import ipm_ref, nlp_ref

    ocp = nlp_ref.UnicycleOCP(N=N)
    X = np.repeat(P[:, None, 0:3], N + 1, axis=1)
    w0 = nlp_ref.join_w(X, np.zeros((P.shape[0], N, 2)))
    iters = []
    P = P.copy()
    import bench

    for _ in range(steps):
        r = ipm_ref.solve_batch(ocp, P, w0=w0, nthreads=1)
        iters.append(r["iters"])
        P[:, 0:3], _ = nlp_ref.F(P[:, 0:3], r["w"][:, 3:5], P[:, 3:6], ocp)
        w0 = bench.shift_np(r["w"], N)
    return P, r, np.array(iters)


def _worker(rank, world, port, B, steps, N, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from mpcx import dist

    r, w = dist.init("gloo")
    assert (r, w) == (rank, world)
    start, stop = dist.shard(B, rank)
    P = dist.config2_inputs(start, stop)
    Pf, res, iters = _closed_loop_shard(P, steps, N)
    S = dist.stats_matrix(Pf, res["w"], res["f"], res["status"], iters)
    S_all = dist.all_gather_stats(S)
    tmax = dist.max_over_ranks(float(rank + 1))
    if rank == 0:
        out.put((S_all, tmax))
    import torch.distributed as tdist

    tdist.barrier()
    tdist.destroy_process_group()


def test_config2_inputs_are_shard_invariant():
    from mpcx import dist

    full = dist.config2_inputs(0, 256)
    parts = [dist.config2_inputs(*dist.shard(64, r)) for r in range(4)]
    assert np.array_equal(np.concatenate(parts), full)
    assert np.all(np.abs(full[84:, 0:2]) <= 5) and np.all(np.abs(full[84:, 2]) <= np.pi / 2)
    assert np.array_equal(full[:84], dist._golden_P())


@pytest.mark.timeout(300)
def test_world_size_2_gloo_matches_single_process():
    from mpcx import dist

    B, steps, N, world = 16, 2, 20, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, steps, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    S_all, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert S_all.shape == (world * B, len(dist.STAT_FIELDS))
    assert tmax == 2.0
    # single-process reference over the same 2B global instances
    P = dist.config2_inputs(0, world * B)
    Pf, res, iters = _closed_loop_shard(P, steps, N)
    S_ref = dist.stats_matrix(Pf, res["w"], res["f"], res["status"], iters)
    assert np.array_equal(S_all, S_ref)  # independent instances: bitwise identical


def test_config4_config5_inputs_shard_invariant():
    from mpcx import dist as mdist

    t0a, x0a, par = mdist.config4_inputs(0, 64, N=10)
    t0b, x0b, _ = mdist.config4_inputs(32, 64, N=10)
    np.testing.assert_array_equal(t0a[32:], t0b)
    np.testing.assert_array_equal(x0a[32:], x0b)
    assert t0a.min() >= 0 and t0a.max() <= 449 and par.shape == (500, 10, 5)
    a = mdist.config5_inputs(0, 40)
    b = mdist.config5_inputs(10, 40)
    np.testing.assert_array_equal(a[10:], b)
    assert np.all(np.abs(a) <= [1, .5, .2, .5])


def test_bench_gpus_flag_launch_plan():
    """`--gpus N` is honoured: under a launcher the world size must equal N; a plain
    `python bench.py --gpus N` starts N ranks itself through torch.distributed.run (loopback
    rendezvous); a mismatch exits non-zero before any GPU call, so no line with another
    n_gpus is ever printed."""
    import bench

    assert bench.launch_plan(1, env={}) == ("run", None)
    assert bench.launch_plan(8, env={"WORLD_SIZE": "8", "RANK": "3"}) == ("run", None)
    plan, argv = bench.launch_plan(4, env={}, n_devices=8)
    assert plan == "spawn"
    assert argv[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in argv and "--master-addr=127.0.0.1" in argv
    assert argv[7].endswith("bench.py")
    for bad in (dict(gpus=4, env={"WORLD_SIZE": "2", "RANK": "0"}), dict(gpus=2, env={"WORLD_SIZE": "1", "RANK": "0"}),
                dict(gpus=4, env={}, n_devices=1), dict(gpus=0, env={})):
        with pytest.raises(SystemExit):
            bench.launch_plan(**bad)
    # one-GPU rehearsal of the multi-rank path (MPCX_FORCE_DEVICE): allowed past the device count
    assert bench.launch_plan(2, env={"MPCX_FORCE_DEVICE": "0"}, n_devices=1)[0] == "spawn"


def test_bench_gpus_mismatch_exits_nonzero():
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_visible_gpu_count_reads_topology_without_hip(tmp_path):
    """bench.py decides its launch plan on mdist.visible_gpu_count(): the KFD topology's GPU
    nodes (gpu_id != 0; CPU nodes have gpu_id 0), capped by *_VISIBLE_DEVICES, no HIP call."""
    from mpcx import dist as mdist

    for i, gid in enumerate([0, 0, 1234, 5678, 91011]):  # two CPU nodes, three GPUs
        d = tmp_path / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{gid}\n")
    assert mdist.visible_gpu_count(str(tmp_path), environ={}) == 3
    assert mdist.visible_gpu_count(str(tmp_path), environ={"HIP_VISIBLE_DEVICES": "0,2"}) == 2
    assert mdist.visible_gpu_count(str(tmp_path), environ={"ROCR_VISIBLE_DEVICES": "1"}) == 1
    assert mdist.visible_gpu_count(str(tmp_path / "missing"), environ={}) is None
