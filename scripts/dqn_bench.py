"""Throughput of the fused DQN consumer (snake_dqn_forward, dqn_kernels.hip) on
one GPU, beside the same network run by PyTorch eager (MIOpen convolutions,
hipBLASLt linears) in fp32 and bf16 on the same observations.

The workload is one forward over the bench's observation batch: 65,536 envs x 4
snakes = 262,144 observations of 11x11x8 (vision_range 5, frame_stack 1), the
network of train_dqn.py:104-151 with random-init weights.

Algorithmic FLOP per observation (multiply-add = 2, unpadded shapes):
  conv_l: 2 * h*w * cout * 9*cin      fc: 2 * in * out
Prints one JSON line: obs/s, ms per forward, TFLOP/s and its fraction of the
2.5 PFLOP/s dense bf16 MFMA peak (MI355X_MICROARCH.md), torch timings.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'marl-snake_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import torch  # noqa: E402

PEAK_BF16 = 2.5e15
PEAK_FP32 = 157.3e12   # MI355X fp32 (vector and matrix)


def flops_per_obs(h, w, c, a):
    p = h * w
    return 2 * (p * 32 * 9 * c + p * 64 * 9 * 32 + p * 64 * 9 * 64 + 64 * p * 256 + 256 * 128 + 128 * a)


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=65536)
    ap.add_argument('--snakes', type=int, default=4)
    ap.add_argument('--vr', type=int, default=5)
    ap.add_argument('--fs', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--no-torch', action='store_true')
    ap.add_argument('--precision', choices=('bf16', 'fp32'), default='bf16')
    args = ap.parse_args()

    from marlenv import SnakeVecEnv
    from marlenv.dqn import DQNForward
    from test_dqn import RefDQN

    torch.manual_seed(0)
    env = SnakeVecEnv(args.envs, num_snakes=args.snakes, seed=0, height=20, width=20,
                      vision_range=args.vr or None, frame_stack=args.fs)   # --vr 0: full 20x20 map
    env.reset()
    g = torch.Generator(device='cuda').manual_seed(0)
    for _ in range(8):
        o, _, _, _ = env.step(torch.randint(0, 3, (args.envs, args.snakes), generator=g, device='cuda',
                                            dtype=torch.int8))
    obs = o.reshape(-1, *o.shape[2:]).contiguous()
    B, h, w, c = obs.shape
    del env
    ref = RefDQN(h, w, c, 3).cuda().eval()
    net = DQNForward(ref, h, w, c, 3, precision=args.precision)
    fpo = flops_per_obs(h, w, c, 3)
    peak = PEAK_BF16 if args.precision == 'bf16' else PEAK_FP32

    ms = timed(lambda: net(obs), args.steps, args.warmup)
    tf = fpo * B / (ms * 1e-3)
    out = {'metric': 'dqn_forward_obs_per_sec', 'value': B / (ms * 1e-3), 'unit': 'obs/s',
           'ms_per_forward': ms, 'batch': B, 'obs_shape': [h, w, c],
           'dtype': 'bf16 (fp32 accumulate)' if args.precision == 'bf16' else 'fp32',
           'flop_per_obs': fpo,
           'roofline': {'bound': 'mfma' if args.precision == 'bf16' else 'fp32 (vector = matrix peak)',
                        'achieved': tf / 1e12, 'peak': peak / 1e12, 'unit': 'TFLOP/s', 'frac': tf / peak}}
    if not args.no_torch:
        with torch.no_grad():
            ms32 = timed(lambda: ref(obs), max(3, args.steps // 4), 2)
            refb = RefDQN(h, w, c, 3).cuda().eval().to(torch.bfloat16)
            refb.load_state_dict({k: v.to(torch.bfloat16) for k, v in ref.state_dict().items()})

            def fb():
                x = obs.permute(0, 3, 1, 2).to(torch.bfloat16)
                x = torch.relu(refb.conv1(x))
                x = torch.relu(refb.conv2(x))
                x = torch.relu(refb.conv3(x))
                x = torch.relu(refb.fc1(x.reshape(B, -1)))
                return refb.fc3(torch.relu(refb.fc2(x)))
            msb = timed(fb, max(3, args.steps // 4), 2)
        out['torch_eager'] = {'fp32_ms': ms32, 'bf16_ms': msb, 'fp32_obs_per_sec': B / (ms32 * 1e-3),
                              'bf16_obs_per_sec': B / (msb * 1e-3)}
        out['speedup_vs_torch_fp32'] = ms32 / ms
        out['speedup_vs_torch_bf16'] = msb / ms
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    t0 = time.time()
    main()
    print('# wall %.1f s' % (time.time() - t0), file=sys.stderr)
