"""The N>1 path on CPU: world_size-2 gloo ranks.

bench.py shards the env batch contiguously over ranks, seeds env i with its
GLOBAL index (SnakeVecEnv env_offset), runs no collective on the step path and
max-reduces the timings. Here two gloo ranks check that the shards tile the batch,
that the max-reduce is the slowest rank's time, and -- with the CPU restatement
standing in for the device env -- that the sharded rollout is identical to the
single-process one (digests all-gathered over gloo).
"""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

KW = dict(num_snakes=4, height=12, width=12, snake_length=3, vision_range=3)
N_TOTAL, STEPS = 6, 25


def rollout_digests(lo, hi, oracle_lib):
    """Per-env digest of a random-action rollout (all-done auto-reset), env i seeded i."""
    from oracle.snake_oracle import OracleEnv
    out = []
    for i in range(lo, hi):
        e = OracleEnv(i, **KW)
        h = hashlib.blake2b(e.reset().tobytes(), digest_size=8)
        rs = np.random.RandomState(1000 + i)
        for _ in range(STEPS):
            obs, rew, done, _ = e.step(rs.randint(0, 3, size=KW['num_snakes']))
            h.update(obs.tobytes())
            h.update(np.asarray(rew, dtype=np.float64).tobytes())
            if np.all(done):
                h.update(e.reset().tobytes())
        out.append(int.from_bytes(h.digest(), 'little') & ((1 << 62) - 1))
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        lo, hi = bench.shard_range(N_TOTAL, world, rank)
        # timings: rank r reports (1 + r, 10 - r); the reduce keeps the slowest per field
        red = bench.reduce_max([1.0 + rank, 10.0 - rank], torch.device('cpu'), dist)
        dig = rollout_digests(lo, hi, None)
        sizes = [None] * world
        dist.all_gather_object(sizes, (lo, hi))
        gathered = [None] * world
        dist.all_gather_object(gathered, dig)
        if rank == 0:
            q.put((sizes, red, [d for g in gathered for d in g]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_shards_match_single_process(oracle):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    sizes, red, digests = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sizes == [(0, 3), (3, 6)]
    assert red == [2.0, 10.0]
    assert digests == rollout_digests(0, N_TOTAL, None)


@pytest.mark.parametrize('n,world', [(65536, 8), (10, 3), (7, 8), (1, 1)])
def test_shard_range_tiles(n, world):
    rs = [bench.shard_range(n, world, r) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_batch_plan_strong_and_weak():
    """BASELINE.json's metric fixes the whole-node batch (65 536 envs over 1 -> 8
    GPUs): cfg3 shards it (strong, 8 192 per GPU at 8 ranks) unless a per-GPU
    batch is asked for; the other presets name a per-GPU share (weak)."""
    for world in (1, 2, 4, 8):
        sc, n = bench.batch_plan('cfg3', None, world, None, None)
        assert (sc, n) == ('strong', 65536)
        assert bench.shard_range(n, world, 0) == (0, 65536 // world)
        assert bench.batch_plan('cfg3', 'weak', world, None, None) == ('weak', 65536 * world)
        assert bench.batch_plan('cfg3', None, world, 1024, None) == ('weak', 1024 * world)
        assert bench.batch_plan('cfg4', None, world, None, None) == ('weak', 32768 * world)
        assert bench.batch_plan('cfg3s8', None, world, None, None) == ('weak', 8192 * world)
        assert bench.batch_plan('cfg5', 'strong', world, None, None) == ('strong', 8192)
        assert bench.batch_plan('cfg2', None, world, None, 1000) == ('strong', 1000)
    assert bench.shard_range(65536, 8, 7) == (57344, 65536)
    with pytest.raises(SystemExit):
        bench.batch_plan('cfg3', 'strong', 8, None, 4)


def test_bench_starts_its_ranks_without_a_launcher(monkeypatch):
    """`bench.py --gpus N` with no WORLD_SIZE runs the same command line under
    torch.distributed.run as a child (no exec, nothing touches the GPU first)
    and exits with its return code."""
    import subprocess
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen['cmd'], seen['env'] = cmd, env
        return Done()
    monkeypatch.setattr(subprocess, 'run', fake_run)
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2', '--dist-backend', 'gloo', '--steps', '3'])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 7
    cmd = seen['cmd']
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert cmd[cmd.index('--nproc-per-node') + 1] == '2' and cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-6:] == ['--gpus', '2', '--dist-backend', 'gloo', '--steps', '3']
    assert os.path.basename(cmd[-7]) == 'bench.py'
    assert seen['env']['MASTER_ADDR'] == '127.0.0.1'
