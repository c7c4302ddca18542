"""The N>1 bench path executed on hardware: two ranks of
bench.main on the one GPU of the box (gloo process group: RCCL refuses two ranks
on one device), launched as child processes through torch.distributed.run
exactly as the driver launches N GPUs. A one-rank launch over RCCL (the
driver's backend) runs the nccl process group, barrier and device-side max-reduce
on the box's one GPU. Each rank steps its contiguous shard
(env i seeded with its global index, actions drawn for the whole batch and
sliced), and the concatenated shard results must equal one process stepping the
whole batch: final grids, MT19937 keys and positions, env records, the last
observation and every env's summed rewards, bit for bit."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run(cmd, tmp_path, name):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    log = tmp_path / f'{name}.log'
    with open(log, 'w') as fp:
        rc = subprocess.run(cmd, cwd=ROOT, env=env, stdout=fp, stderr=subprocess.STDOUT, timeout=300).returncode
    text = log.read_text()
    assert rc == 0, f'{name} exited {rc}:\n{text[-3000:]}'
    return [json.loads(x) for x in text.splitlines() if x.startswith('{"metric"')]


@pytest.mark.timeout(600)
@pytest.mark.parametrize('config,per,bg', [('cfg3', 768, -1), ('cfg3', 768, 0), ('cfg5', 96, 0)])
def test_two_ranks_equal_one_process(tmp_path, config, per, bg):
    """bg: --spawn-background (0 automatic: on for both of these small shards,
    -1 the in-step spawn-ahead of large 20x20 shards)."""
    if not os.path.exists(os.path.join(ROOT, 'marl-snake_amd', 'marlenv', 'libsnake_amd.so')):
        pytest.fail('libsnake_amd.so not built')
    common = ['--steps', '40', '--warmup', '10', '--no-cpu-baseline', '--timing-stride', '4',
              '--global-actions', '--config', config, '--spawn-background', str(bg)]
    two = tmp_path / 'two'
    lines = _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                  '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), 'bench.py', '--gpus', '2',
                  '--dist-backend', 'gloo', '--envs-per-gpu', str(per), '--dump-dir', str(two)] + common,
                 tmp_path, 'two')
    assert len(lines) == 1, 'rank 0 prints exactly one JSON line'
    line = lines[0]
    assert line['n_gpus'] == 2 and line['config']['num_envs'] == 2 * per and line['scaling'] == 'weak'
    assert line['value'] > 0 and line['steps'] == 40
    one = tmp_path / 'one'
    lines1 = _run([sys.executable, 'bench.py', '--envs-per-gpu', str(2 * per), '--dump-dir', str(one)] + common,
                  tmp_path, 'one')
    assert len(lines1) == 1 and lines1[0]['n_gpus'] == 1
    full = np.load(one / 'rank0.npz')
    parts = [np.load(two / f'rank{r}.npz') for r in range(2)]
    assert [(int(p['lo']), int(p['hi'])) for p in parts] == [(0, per), (per, 2 * per)]
    for key in ('grids', 'mt', 'mt_pos', 'env', 'obs', 'rew_sum'):
        # (all eight env record words: bench.py dumps SnakeVecEnv.env_records(),
        # the spawn-ahead status word in its canonical form)
        cat, ref = np.concatenate([p[key] for p in parts]), full[key]
        assert cat.tobytes() == ref.tobytes(), key
    if config == 'cfg3':   # the rollout went through episode ends (auto-resets on both ranks)
        assert all(int(p['env'][:, 1].min()) < 50 for p in parts)


@pytest.mark.timeout(600)
def test_rccl_rank_equals_plain_process(tmp_path):
    """bench.py under torch.distributed.run with the nccl (RCCL) backend: one rank
    on the box's GPU, the same rollout as the plain process, one JSON line whose
    time went through the device-side all_reduce(MAX)."""
    common = ['--steps', '30', '--warmup', '10', '--no-cpu-baseline', '--timing-stride', '4',
              '--global-actions', '--config', 'cfg3', '--envs-per-gpu', '1024',
              '--spawn-background', '-1']   # (in-step spawn-ahead: the status word is exact too)
    r = tmp_path / 'rccl'
    lines = _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                  '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), 'bench.py', '--gpus', '1',
                  '--dist-backend', 'nccl', '--dump-dir', str(r)] + common, tmp_path, 'rccl')
    assert len(lines) == 1 and lines[0]['n_gpus'] == 1 and lines[0]['value'] > 0
    assert lines[0]['process_group'] == 'nccl'
    one = tmp_path / 'one'
    _run([sys.executable, 'bench.py', '--dump-dir', str(one)] + common, tmp_path, 'one')
    a, b = np.load(r / 'rank0.npz'), np.load(one / 'rank0.npz')
    for key in ('grids', 'mt', 'mt_pos', 'env', 'obs', 'rew_sum'):
        assert a[key].tobytes() == b[key].tobytes(), key


@pytest.mark.timeout(600)
def test_strong_scaling_self_launched(tmp_path):
    """`bench.py --gpus 2` with no launcher in front (no WORLD_SIZE): bench.py
    starts its two ranks itself under torch.distributed.run and relays rank 0's
    line. Strong scaling: the fixed whole-job batch (--num-envs) is split into
    two shards, and their concatenated results equal one process stepping the
    whole batch -- every env record word included (the spawn-ahead status word
    is dumped in its canonical form, SnakeVecEnv.env_records)."""
    n = 1536
    common = ['--steps', '40', '--warmup', '10', '--no-cpu-baseline', '--timing-stride', '4',
              '--global-actions', '--config', 'cfg3', '--num-envs', str(n)]
    two = tmp_path / 'two'
    lines = _run([sys.executable, 'bench.py', '--gpus', '2', '--dist-backend', 'gloo', '--dump-dir', str(two)] + common,
                 tmp_path, 'two')
    assert len(lines) == 1, 'rank 0 prints exactly one JSON line'
    line = lines[0]
    assert line['n_gpus'] == 2 and line['scaling'] == 'strong' and line['process_group'] == 'gloo'
    assert line['config']['num_envs'] == n and line['config']['envs_per_gpu'] == n // 2
    one = tmp_path / 'one'
    lines1 = _run([sys.executable, 'bench.py', '--dump-dir', str(one)] + common, tmp_path, 'one')
    assert len(lines1) == 1 and lines1[0]['n_gpus'] == 1 and lines1[0]['scaling'] == 'strong'
    full = np.load(one / 'rank0.npz')
    parts = [np.load(two / f'rank{r}.npz') for r in range(2)]
    assert [(int(p['lo']), int(p['hi'])) for p in parts] == [(0, n // 2), (n // 2, n)]
    for key in ('grids', 'mt', 'mt_pos', 'env', 'obs', 'rew_sum'):
        cat = np.concatenate([p[key] for p in parts])
        assert cat.tobytes() == full[key].tobytes(), key
