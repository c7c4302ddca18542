#!/usr/bin/env python3
"""Throughput of the batched multi-snake env step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg3s8|cfg4|cfg5]
                    [--scaling strong|weak]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

--gpus N > 1 without a launcher (no WORLD_SIZE in the environment) starts the N
ranks itself: `python -m torch.distributed.run --nproc-per-node N` on this same
command line, as a child process started before anything touches the GPU; rank
0's JSON line is relayed (the children share stdout) and so is the return code.

Workload (BASELINE.json metric, config 3 by default): 65 536 envs of 20x20
grids, 4 snakes, vision_range=5, frame_stack=1, snake_length=3, default
rewards, uniform random actions in {0,1,2} drawn up front on the device (seed
12345), all-done auto-reset inside the step. Env i is seeded with its GLOBAL
index, so ranks hold disjoint contiguous shards of one batch (no collective on
the step path; the only collectives are the timing barrier and max-reduce).
The metric's batch is fixed ("whole-node, 65536 envs ... 1->8 GPU"), so cfg3
scales STRONG by default: 65 536 envs in all, 65 536 / N per GPU (8 192 at 8
GPUs). --scaling weak keeps the per-GPU batch instead (65 536 per GPU).
--config picks BASELINE.json's other configs (their presets are the per-GPU
share of the 8-GPU configuration, weak scaling by default):
  cfg2    4 096 envs/GPU, 20x20, 4 snakes, full-map observation
  cfg3    65 536 envs in all (default), 20x20, 4 snakes, vision_range 5
  cfg3s8  8 192 envs/GPU: cfg3's per-GPU shard at 8 GPUs, on one GPU
  cfg4    32 768 envs/GPU (262 144 over 8 GPUs), 20x20, 4 snakes, vision_range 5
  cfg5    8 192 envs/GPU (65 536 over 8 GPUs), 40x40, 8 snakes, vision_range 5, frame_stack 4

A step = one SnakeVecEnv.step() over the GPU's whole batch. The timed region is
exactly K steps between barrier + synchronize on both sides; value = all envs of
all ranks x K / the slowest rank's time.

A step is two launches on the caller's stream (include/snake_env.h snake_step):
k_logic (rules, all envs), then k_post, whose first blocks are the reset workers
(the step's auto-resets, then the spawn-ahead attempts: next resets'
permutations drawn early) and the rest the observations of every other env. On
boards of more than 8 192 spawn poses (cfg5) it is k_post_lean (resets-only
workers + four-wave lean encodes) and the spawn-ahead attempts run in k_spawn on
a background stream the step never waits for.

The JSON line also carries:
  roofline     -- the kernel that moves the bulk of SURVEY.md 8(d)'s bytes:
                  k_post (k_post_lean at cfg5), per launch (N - resets) x (S*h*w*8*fs obs
                  write + fs*H*W frame reads) [+ for k_post, per reset 2 MT keys +
                  fs*H*W + S*h*w*8*fs, per spawn-ahead attempt 2 MT keys + the
                  pose indices] / its average duration, timed by the library's HIP
                  timing events on its own stream during the timed region
                  (snake_timing_enable; every --timing-stride-th step, default
                  max(1, min(32, steps // 4)) so that >= 4 launches are averaged),
                  against the 8 TB/s HBM peak; `traffic` is null (the HBM bytes of
                  a launch come from rocprofv3 PMC passes, committed under
                  profiles/, which a plain run cannot read).
  step_roofline -- the whole step against the same peak: B = S*h*w*8*fs +
                  (fs+1)*H*W + 10*S bytes per env-step x envs /
                  ms_per_step.
  kernels      -- average device ms per launch of each step kernel (same events).
  cpu_baseline -- rank 0 at N=1: the CPU restatement (oracle/, a C port of the
                  reference SnakeEnv) on every available host core (one process
                  per core, at most 16: the box's CPU share), a bounded sample of
                  the same workload, run BEFORE the GPU is touched; plus the
                  reference-equivalent rate from profiles/cpu_ratio.json (the
                  C-to-reference speed ratio measured where the reference runs,
                  scripts/cpu_ratio.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, 'marl-snake_amd'), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = 'env-steps/sec whole-node, 65536×(20×20, 4 snakes), random actions; 1→8 GPU'
HBM_PEAK_GBS = 8000.0


def shard_range(n_total, world, rank):
    """Contiguous env range [lo, hi) of one rank."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def reduce_max(values, device, dist=None):
    """Element-wise max over ranks (the slowest rank's times); identity at world 1."""
    if dist is None:
        return list(values)
    import torch
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def algorithmic_bytes(S, h, w, fs, H, W):
    """obs write + grid ring read/write + actions/rewards/dones."""
    return S * h * w * 8 * fs + (fs + 1) * H * W + S * (1 + 8 + 1)


def encode_bytes(S, h, w, fs, H, W):
    """k_encode per encoded env: the stacked-frame observation written + the fs
    grid frames read."""
    return S * h * w * 8 * fs + fs * H * W


MT_KEY_BYTES = 624 * 4


def reset_bytes(S, h, w, fs, H, W):
    """One auto-reset (do_reset from a ready spawn-ahead record): the MT key read
    from the record and stored back, the fs fresh frames and the first
    observation written."""
    return 2 * MT_KEY_BYTES + fs * H * W + S * h * w * 8 * fs


def spawn_bytes(S):
    """One spawn-ahead attempt: the env's MT key read, the record (key, position,
    S pose indices) written."""
    return 2 * MT_KEY_BYTES + 4 * (1 + S)


PRESETS = {   # BASELINE.json configs (per GPU)
    'cfg2': dict(envs_per_gpu=4096, height=20, width=20, num_snakes=4, vision_range=0, frame_stack=1),
    'cfg3': dict(envs_per_gpu=65536, height=20, width=20, num_snakes=4, vision_range=5, frame_stack=1),
    'cfg3s8': dict(envs_per_gpu=8192, height=20, width=20, num_snakes=4, vision_range=5, frame_stack=1),
    'cfg4': dict(envs_per_gpu=32768, height=20, width=20, num_snakes=4, vision_range=5, frame_stack=1),
    'cfg5': dict(envs_per_gpu=8192, height=40, width=40, num_snakes=8, vision_range=5, frame_stack=4),
}
# the whole-node batch of the configs whose batch is fixed (strong scaling by
# default): BASELINE.json's metric, 65 536 envs over 1 -> 8 GPUs
STRONG_TOTAL = {'cfg3': 65536}


def batch_plan(config, scaling, world, envs_per_gpu, num_envs):
    """(scaling, n_total) of a run: strong keeps the whole batch fixed (num_envs,
    else the config's STRONG_TOTAL) and shards it over the ranks; weak runs
    envs_per_gpu on every rank. Default: strong for the metric's config unless
    the per-GPU batch was given, else weak."""
    if scaling is None:
        scaling = 'strong' if (num_envs is not None or (config in STRONG_TOTAL and envs_per_gpu is None)) else 'weak'
    if scaling == 'strong':
        n = num_envs if num_envs is not None else STRONG_TOTAL.get(config, PRESETS[config]['envs_per_gpu'])
        if n < world:
            raise SystemExit(f'--scaling strong: {n} envs cannot be sharded over {world} ranks')
        return scaling, n
    per = envs_per_gpu if envs_per_gpu is not None else PRESETS[config]['envs_per_gpu']
    return scaling, per * world


def launch_ranks(n, argv):
    """--gpus N without a launcher: run this command line under
    torch.distributed.run (N ranks on this node, rendezvous on 127.0.0.1) as a
    child process and return its exit code. Called before torch touches the GPU;
    the ranks inherit stdout, so rank 0's JSON line reaches the caller as is."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    return subprocess.run(cmd, env=env).returncode


def _cpu_worker(args):
    env_kw, num_snakes, seconds, wid = args
    import time as _t
    from oracle.snake_oracle import rollout
    n, steps, t0 = 0, 32, _t.perf_counter()
    while _t.perf_counter() - t0 < seconds:
        n += rollout(16, 1000 * wid, steps, act_seed=12345 + wid, num_snakes=num_snakes, **env_kw)
        steps = min(2 * steps, 2048)
    return n, _t.perf_counter() - t0


def cpu_baseline(env_kw, num_snakes, seconds, ratio_key):
    """The C restatement of the reference step (oracle/so_rollout: 16 envs per
    process, random actions, all-done resets) on every available core, one
    forked process per core. Runs before the GPU is initialised."""
    import multiprocessing as mp
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    ctx = mp.get_context('fork')
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(env_kw, num_snakes, seconds, w) for w in range(cores)])
    n = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    out = dict(value=round(n / el, 1), unit='env-steps/s', cores=cores, kind='port',
               sample=f'{cores} processes x 16 envs, {n} env-steps incl. auto-resets in {el:.1f} s, '
                      'oracle/snake_oracle.c so_rollout (serial C restatement of SnakeEnv.step/reset)')
    try:
        with open(os.path.join(ROOT, 'profiles', 'cpu_ratio.json')) as fp:
            r = json.load(fp)[ratio_key]
        out['port_over_reference_1core'] = r['port_over_reference']
        out['reference_equivalent'] = round(n / el / r['port_over_reference'], 1)
        out['reference_1core_measured'] = r['reference_env_steps_per_s_1core']
        out['ratio_source'] = 'profiles/cpu_ratio.json (scripts/cpu_ratio.py, measured in the build container)'
    except (OSError, ValueError, KeyError):
        pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=200)
    ap.add_argument('--config', choices=sorted(PRESETS), default='cfg3')
    ap.add_argument('--envs-per-gpu', type=int, default=None,
                    help='per-GPU batch (weak scaling; default: the preset\'s)')
    ap.add_argument('--num-envs', type=int, default=None,
                    help='whole-job batch, sharded over the ranks (strong scaling)')
    ap.add_argument('--scaling', choices=('strong', 'weak'), default=None,
                    help='strong: a fixed whole-job batch (default for cfg3, the metric\'s 65 536 envs); '
                         'weak: a fixed per-GPU batch (default for the other presets)')
    ap.add_argument('--height', type=int, default=None)
    ap.add_argument('--width', type=int, default=None)
    ap.add_argument('--num-snakes', type=int, default=None)
    ap.add_argument('--vision-range', type=int, default=None)
    ap.add_argument('--frame-stack', type=int, default=None)
    ap.add_argument('--spawn-background', type=int, default=0,
                    help='snake_cfg.spawn_background: 0 automatic (boards over 8 192 spawn poses, batches '
                         'of up to 8 192 envs and 64 MiB of observations), 1 on, -1 off')
    ap.add_argument('--spawn-ahead', type=int, default=0,
                    help='snake_cfg.spawn_ahead: 0 default threshold, -1 off, k: envs with at most k live snakes')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--dist-backend', choices=('nccl', 'gloo'), default='nccl',
                    help='process group of the timing barrier / max-reduce (gloo: CPU tensors; '
                         'lets several ranks share one GPU, e.g. the two-rank test on a one-GPU box)')
    ap.add_argument('--global-actions', action='store_true',
                    help="every rank draws the WHOLE batch's actions and takes its shard's rows, so "
                         'any world size replays the same rollout (check runs; the default draws per rank)')
    ap.add_argument('--dump-dir', default=None,
                    help='write rank<r>.npz with the shard range, final grids, MT keys/positions, '
                         'env records, the last step\'s obs and each env\'s summed rewards')
    ap.add_argument('--timing-warm', type=int, default=4,
                    help='time (and drop) the last k warmup steps so the event pool is filled before the timed region')
    ap.add_argument('--timing-stride', type=int, default=None,
                    help='bracket the kernels of every k-th timed step with timing events '
                         '(0: none; default max(1, min(32, steps // 4)), so at least 4 launches are '
                         'averaged; a timed step costs ~1-2 us more: 0.1034 ms per step at stride 32 vs 0.1025 untimed, cfg3)')
    args = ap.parse_args()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    scaling, n_total = batch_plan(args.config, args.scaling, world, args.envs_per_gpu, args.num_envs)
    for k, v in PRESETS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    rank = int(os.environ.get('RANK', '0'))
    env_kw = dict(height=args.height, width=args.width, snake_length=3,
                  vision_range=args.vision_range or None, frame_stack=args.frame_stack)
    S = args.num_snakes
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        key = None
        if (args.height, args.width, S, args.frame_stack) == (20, 20, 4, 1) and args.vision_range in (0, 5):
            key = 'cfg3_20x20_s4_vr5' if args.vision_range else 'cfg2_20x20_s4_full'
        cpu = cpu_baseline(env_kw, S, args.cpu_seconds, key)

    import torch
    import torch.distributed as dist

    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    # under torch.distributed.run even one rank joins the process group, so the
    # RCCL barrier / device-side max-reduce of the N-GPU line runs on a 1-GPU box
    distributed = world > 1 or 'LOCAL_WORLD_SIZE' in os.environ
    ordinal = local_rank % max(1, torch.cuda.device_count())   # ranks beyond the GPUs share them (gloo only)
    if distributed:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(ordinal)
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', ordinal))
        else:
            dist.init_process_group('gloo')
    device = torch.device('cuda', ordinal if distributed else torch.cuda.current_device())
    red_device = device if args.dist_backend == 'nccl' else torch.device('cpu')

    from marlenv import SnakeVecEnv
    from marlenv import _native

    lo, hi = shard_range(n_total, world, rank)
    per = shard_range(n_total, world, 0)[1]   # (the largest shard: rank 0's)
    venv = SnakeVecEnv(hi - lo, num_snakes=S, device=device, seed=0, env_offset=lo,
                       spawn_background=args.spawn_background, spawn_ahead=args.spawn_ahead, **env_kw)
    venv.reset()
    gen = torch.Generator(device=device)
    n_act = args.warmup + args.steps
    if args.global_actions:
        gen.manual_seed(12345)
        actions = torch.randint(0, 3, (n_act, n_total, S), generator=gen, device=device,
                                dtype=torch.int8)[:, lo:hi].contiguous()
    else:
        gen.manual_seed(12345 + rank)
        actions = torch.randint(0, 3, (n_act, hi - lo, S), generator=gen, device=device, dtype=torch.int8)
    rsum = torch.zeros((hi - lo, S), dtype=torch.float64, device=device) if args.dump_dir else None

    # (outputs are dropped at once unless --dump-dir sums them: holding a step's
    # outputs while the next step runs makes the allocator alternate between two
    # observation buffers; measured +4 us per step at cfg3)
    out = None
    L = _native.lib()
    for t in range(args.warmup):
        # the last --timing-warm warmup steps are timed and their timings dropped:
        # the library's event pool then holds the events the timed steps use
        # (creating them inside the timed region stalls the first timed steps)
        warm = t >= args.warmup - args.timing_warm
        if warm:
            _native.timing_enable(True, L)
        if rsum is None:
            venv.step(actions[t])
        else:
            out = venv.step(actions[t])
            rsum += out[1]
        if warm:
            _native.timing_enable(False, L)
    torch.cuda.synchronize(device)

    for k in ('k_logic', 'k_autoreset', 'k_encode', 'k_post', 'k_spawn', 'resets', 'resets_timed', 'spawn_hits',
              'spawn_jobs', 'spawn_void', 'reset_partial'):
        _native.timing_read(k, L)                      # drop anything from the warmup
    stride = args.timing_stride if args.timing_stride is not None else max(1, min(32, args.steps // 4))
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for t in range(args.steps):
        timed = stride > 0 and t % stride == 0
        if timed:
            _native.timing_enable(True, L)
        if rsum is None:
            venv.step(actions[args.warmup + t])
        else:
            out = venv.step(actions[args.warmup + t])
            rsum += out[1]
        if timed:
            _native.timing_enable(False, L)
    torch.cuda.synchronize(device)
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern = {}
    for k in ('k_logic', 'k_autoreset', 'k_encode', 'k_post', 'k_spawn'):
        ms, n = _native.timing_read(k, L)
        kern[k] = ms / max(n, 1)
    resets = _native.timing_read('resets', L)[1]              # every timed step
    # counted on the event-timed steps only, the steps the kernel times come from:
    # the auto-resets, the resets served from a spawn-ahead record, the attempts
    n_timed = len(range(0, args.steps, stride)) if stride > 0 else 0
    resets_t = _native.timing_read('resets_timed', L)[1]
    sp_hits = _native.timing_read('spawn_hits', L)[1]
    sp_jobs = _native.timing_read('spawn_jobs', L)[1]
    sp_void = _native.timing_read('spawn_void', L)[1]
    rs_part = _native.timing_read('reset_partial', L)[1]
    # per launch on the event-timed steps (all steps when no step is timed)
    rps_t = resets_t / n_timed if n_timed else resets / args.steps

    red = reduce_max([elapsed] + list(kern.values()), red_device, dist if distributed else None)
    elapsed, kern = red[0], dict(zip(kern, red[1:]))

    lay = venv.layout
    B = algorithmic_bytes(S, lay.obs_h, lay.obs_w, args.frame_stack, args.height, args.width)
    Be = encode_bytes(S, lay.obs_h, lay.obs_w, args.frame_stack, args.height, args.width)
    encoded_per_launch = (hi - lo) - rps_t
    if kern['k_post'] > 0:
        # the shared phase as one launch (k_post: reset workers + encodes): its
        # bytes are the encodes', the resets' and the spawn-ahead attempts'
        rk, rk_ms = 'k_post', kern['k_post']
        # (with background spawn-ahead the attempts are k_spawn's, not k_post's)
        jobs_per_step = sp_jobs / n_timed if n_timed and kern['k_spawn'] == 0 else 0.0
        launch_bytes = (Be * encoded_per_launch
                        + reset_bytes(S, lay.obs_h, lay.obs_w, args.frame_stack, args.height, args.width)
                        * rps_t + spawn_bytes(S) * jobs_per_step)
    else:
        rk, rk_ms = 'k_encode', kern['k_encode']
        launch_bytes = Be * encoded_per_launch
    achieved = launch_bytes / (rk_ms * 1e-3) / 1e9 if rk_ms > 0 else float('nan')
    value = n_total * args.steps / elapsed
    step_gbs = B * (hi - lo) / (elapsed / args.steps) / 1e9
    preset = PRESETS[args.config]
    as_preset = all(getattr(args, k) == v for k, v in preset.items() if k != 'envs_per_gpu')
    as_preset = as_preset and n_total == (STRONG_TOTAL.get(args.config, preset['envs_per_gpu']) if scaling == 'strong'
                                          else preset['envs_per_gpu'] * world)
    name = args.config if as_preset else 'custom'
    shard = f'{n_total} envs in all, {per} per GPU' if scaling == 'strong' else f'{per} envs/GPU'
    workload = (f'{name}: {shard} x ({args.height}x{args.width}, {S} snakes, '
                f'vision_range={args.vision_range or None}, frame_stack={args.frame_stack}), '
                'random actions, all-done auto-reset in the step')
    line = {
        'metric': METRIC,
        'value': round(value, 1),
        'unit': 'env-steps/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': scaling,
        'vs_baseline': None,
        'dtype': 'u8',
        'data': 'synthetic (uniform random actions, seeded MT19937 envs)',
        'config': {'workload': workload, 'num_envs': n_total, 'envs_per_gpu': per,
                   'height': args.height, 'width': args.width, 'num_snakes': S,
                   'vision_range': args.vision_range, 'frame_stack': args.frame_stack,
                   'snake_length': 3, 'parallelism': f'env-shard x{world}'},
        'process_group': args.dist_backend if distributed else None,
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                     'traffic': None, 'kernel': rk, 'kernel_ms': round(rk_ms, 4), 'timed_launches': n_timed,
                     'algorithmic_bytes_per_launch': round(launch_bytes),
                     'bytes_per_encoded_env': Be},
        'step_roofline': {'achieved': round(step_gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                          'frac': round(step_gbs / HBM_PEAK_GBS, 4), 'bytes_per_env_step': B},
        'kernels': {k: round(v, 4) for k, v in kern.items()},
        'resets_per_step': round(resets / args.steps, 1),
        'resets_per_timed_step': round(rps_t, 1),
        # every env is reset at once before the warmup; its episodes end ~20-120
        # steps later, so a short warmup times that wave of resets, not the steady
        # rate (~1 036 per step at cfg3 past ~200 steps)
        'regime': ('steady (warmup >= 200 steps after env.reset())' if args.warmup >= 200 else
                   f'post-reset transient (steps {args.warmup}-{args.warmup + args.steps} after env.reset())'),
        'spawn_ahead': ({'hits_per_step': round(sp_hits / n_timed, 1),
                         'jobs_per_step': round(sp_jobs / n_timed, 1),
                         'jobs_per_served_reset': round(sp_jobs / max(sp_hits, 1), 3),
                         'ready_voided_per_step': round(sp_void / n_timed, 1),
                         'resets_from_partial_per_step': round(rs_part / n_timed, 2),
                         'resets_without_record_per_step': round((resets_t - sp_hits - rs_part) / n_timed, 2),
                         'hit_rate': round(sp_hits / max(resets_t, 1), 4)}
                        if n_timed else None),
        'cpu_baseline': None,
    }
    line['cpu_baseline'] = cpu
    if args.dump_dir:
        import numpy as np
        os.makedirs(args.dump_dir, exist_ok=True)
        venv.sync()   # (after the last background spawn kernel)
        keys, pos = venv.mt_state()
        np.savez(os.path.join(args.dump_dir, f'rank{rank}.npz'), lo=lo, hi=hi, world=world,
                 grids=venv.grids().cpu().numpy(), mt=keys.cpu().numpy(), mt_pos=pos.cpu().numpy(),
                 env=venv.env_records().cpu().numpy(), obs=out[0].cpu().numpy(),
                 rew_sum=rsum.cpu().numpy())
    if rank == 0:
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
