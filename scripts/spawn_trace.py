#!/usr/bin/env python3
"""Record the per-env, per-step inputs of the spawn-ahead queuing decision
(k_logic, snake_kernels.hip) on the bench workload, for the offline policy
study in scripts/spawn_policy.py. GPU only (SnakeVecEnv, the product path).

Per env and step, after the step's transition, one uint16:
  bits 0-2   live snakes (0 = the episode ended this step)
  bit  3     the step drew from the env's MT19937 (a fruit respawn: it voids a
             ready spawn-ahead record, snake_env.py:376-379)
  bits 4-7   min Manhattan distance from a live head to a fruit (capped at 15)
  bits 8-14  prod over live snakes of the number of their 3 moves that can kill
             them next step (wall / body / head cell, a cell another live snake
             can also enter, the tail of a snake that can eat): 0 = the
             episode cannot end next step (snake_env.py:521-546)

    python scripts/spawn_trace.py --config cfg3 --steps 600 --envs 32768 --out gpurun_out/trace_cfg3.npz
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'marl-snake_amd'))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cfg3')
    ap.add_argument('--steps', type=int, default=600)
    ap.add_argument('--envs', type=int, default=None)
    ap.add_argument('--out', required=True)
    args = ap.parse_args()
    import numpy as np
    import torch
    from bench import PRESETS
    from marlenv import SnakeVecEnv
    p = dict(PRESETS[args.config])
    N = args.envs or p['envs_per_gpu']
    S, H, W = p['num_snakes'], p['height'], p['width']
    dev = torch.device('cuda', 0)
    venv = SnakeVecEnv(N, num_snakes=S, device=dev, seed=0, height=H, width=W, snake_length=3,
                       vision_range=p['vision_range'] or None, frame_stack=p['frame_stack'])
    venv.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(12345)
    rr = torch.arange(H, device=dev, dtype=torch.int16).view(1, 1, H, 1)
    cc = torch.arange(W, device=dev, dtype=torch.int16).view(1, 1, 1, W)
    # moves 0 keep, 1 left (+3), 2 right (+1) of direction d (UP, RIGHT, DOWN, LEFT)
    DR = torch.tensor([-1, 0, 1, 0], device=dev)
    DC = torch.tensor([0, 1, 0, -1], device=dev)
    turn = torch.tensor([0, 3, 1], device=dev)
    trace = torch.empty((args.steps, N), dtype=torch.int16, device=dev)
    _, pos0 = venv.mt_state()
    pos0 = pos0.clone()
    for t in range(args.steps):
        a = torch.randint(0, 3, (N, S), generator=gen, device=dev, dtype=torch.int8)
        _, _, done, info = venv.step(a)
        ep = info['episode_done']
        _, pos1 = venv.mt_state()
        drew = (pos1 != pos0) & ~ep
        pos0 = pos1.clone()
        am = (S - done.sum(1)).to(torch.int16)
        am = torch.where(ep, torch.zeros_like(am), am)
        tab = venv.snake_table().long()
        alive = tab[..., 5].bool()
        g = venv.grids()
        fruit = (g == 2).view(N, 1, H, W)
        hr = tab[..., 0].to(torch.int16).view(N, S, 1, 1)
        hc = tab[..., 1].to(torch.int16).view(N, S, 1, 1)
        d = (rr - hr).abs() + (cc - hc).abs()
        d = torch.where(fruit, d, torch.full_like(d, 99)).view(N, S, -1).amin(2)
        d = torch.where(alive, d, torch.full_like(d, 99)).amin(1).clamp(max=15)
        # next-step danger: the three target cells of every live snake
        nd = (tab[..., 4:5] + turn.view(1, 1, 3)) & 3                       # (N, S, 3)
        tcell = (tab[..., 0:1] + DR[nd]) * W + tab[..., 1:2] + DC[nd]
        tcell = torch.where(alive.unsqueeze(-1), tcell, torch.full_like(tcell, -1 - 0))
        gv = torch.gather(g.view(N, -1).long(), 1, tcell.clamp(min=0).view(N, -1)).view(N, S, 3)
        code, owner = gv % 10, gv // 10
        dead = (code == 1) | (code == 3) | (code == 4)
        can_eat = ((code == 2) & alive.unsqueeze(-1)).any(-1)              # (N, S)
        dead |= (code == 5) & torch.gather(can_eat, 1, owner.clamp(max=S - 1).view(N, -1)).view(N, S, 3)
        # head-on: a target another live snake can also move to
        flat = tcell.view(N, 1, 1, S * 3)
        same = (tcell.unsqueeze(-1) == flat) & alive.view(N, 1, 1, S).repeat_interleave(3, -1).view(N, 1, 1, S * 3)
        other = torch.arange(S, device=dev).repeat_interleave(3).view(1, 1, 1, S * 3) != \
            torch.arange(S, device=dev).view(1, S, 1, 1)
        dead |= (same & other).any(-1) & alive.unsqueeze(-1)
        nk = dead.sum(-1)                                                   # (N, S)
        prod = torch.where(alive, nk, torch.ones_like(nk)).prod(1)
        prod = torch.where(am > 0, prod, torch.zeros_like(prod)).clamp(max=127)
        trace[t] = (am | (drew.to(torch.int16) << 3) | (d << 4) | (prod.to(torch.int16) << 8)).to(torch.int16)
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    np.savez_compressed(args.out, trace=trace.cpu().numpy().view(np.uint16), S=S, H=H, W=W, N=N)
    print('wrote', args.out, tuple(trace.shape))


if __name__ == '__main__':
    main()
