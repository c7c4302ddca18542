"""SnakeVecEnv: N independent SnakeEnv instances stepped by one HIP launch.

Replaces the reference's process-level vectorisation (gym AsyncVectorEnv over
forked SnakeEnv workers, marlenv/marlenv/wrappers.py:203-223) with one
64-lane wavefront per env on the GPU. State and outputs are PyTorch-ROCm
tensors; the kernels are reached through the C-ABI of include/snake_env.h.

Semantics per env are exactly the reference SnakeEnv's (bit-identical grids,
dones and float64 rewards); env i uses its own MT19937 seeded with
``seed + env_offset + i`` (np.random.seed semantics), so a shard of a larger
batch reproduces the same trajectories as the full batch.

Auto-reset (``autoreset=True``, the default): when every done of an env is True
the env is reset inside the same launch and the returned obs is the reset
observation, while rewards/dones/info are the terminal ones -- the worker
semantics of wrappers.py:139-145 (reset on ``all(done)``). ``autoreset='every_step'``
reproduces gym 0.23.1's worker that make_snake actually runs (wrappers.py:212):
every env is reset after every step (rewards/dones/info of the step, the reset obs).
"""
import ctypes
import sys

import numpy as np

from . import spaces
from ._native import SnakeLayout, SnakeOut, SnakeState, check, lib
from .config import build_cfg


def _torch():
    import torch
    return torch


def _raw_stream(index):
    """hipStream_t of the current stream of device `index` (0 = the null stream)."""
    import torch
    return torch._C._cuda_getCurrentRawStream(index)


def _current_device():
    import torch
    return torch._C._cuda_getDevice()


def torch_cuda_alive():
    """False during interpreter shutdown (no library calls from finalizers then;
    `sys` is the module-level binding: an import there fails once meta_path is gone)."""
    return not sys.is_finalizing()


_INFO_KEYS = ('episode_done', 'rank', 'episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills',
              'error')


class _StepInfo(dict):
    """info of one SnakeVecEnv.step: a dict whose tensors are views of the step's
    output slab, made when first read (most callers never read most of them).
    The fills run on the stream the step was enqueued on (its raw handle,
    `_stream`), whatever stream is current at the read; pickling / deepcopy give
    a plain dict of the tensors."""
    __slots__ = ('_env', '_slab', '_es', '_stream')

    def __init__(self, env, slab, stream):
        dict.__init__(self, dict.fromkeys(_INFO_KEYS))
        self._env, self._slab, self._es, self._stream = env, slab, None, stream

    def _make(self, k):
        # rank / ep_stats are stored only where the episode ended (include/snake_env.h
        # snake_out): zeros elsewhere are filled in here, when first read
        env, slab = self._env, self._slab
        if k == 'episode_done':
            return env._view(slab, 'ep_done')
        if k == 'error':
            return env._view(slab, 'err')
        ended = self['episode_done'].view(-1, 1)
        torch = _torch()
        st = None
        if _raw_stream(env._dev_index) == self._stream:
            ctx = torch.cuda.device(env.device)           # (already the step's stream)
        else:
            st = (torch.cuda.default_stream(env.device) if not self._stream
                  else torch.cuda.ExternalStream(self._stream, device=env.device))
            ctx = torch.cuda.stream(st)
        with ctx:
            if k == 'rank':
                out = env._view(slab, 'rank').masked_fill(~ended, 0)
            else:
                if self._es is None:
                    self._es = env._view(slab, 'ep_stats').masked_fill(~ended.view(-1, 1, 1), 0.0)
                out = self._es
        if st is not None:
            # filled on the step's stream, read on the caller's current one: that
            # stream waits for the fill, and the allocator keeps the block until
            # the current stream's work on it is done
            cur = torch.cuda.current_stream(env.device)
            cur.wait_stream(st)
            out.record_stream(cur)
        if k == 'rank':
            return out
        return out[:, ('episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills').index(k)]

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        if v is None:
            v = self._make(k)
            dict.__setitem__(self, k, v)
        return v

    def __reduce__(self):
        return (dict, (self.copy(),))

    def __deepcopy__(self, memo):
        import copy
        return copy.deepcopy(self.copy(), memo)

    def get(self, k, default=None):
        return self[k] if k in self else default

    def __iter__(self):              # (not dict's: dict(info) / {**info} then go through __getitem__)
        return iter(list(dict.keys(self)))

    def keys(self):
        return dict.keys(self)

    def values(self):
        return [self[k] for k in self]

    def items(self):
        return [(k, self[k]) for k in self]

    def copy(self):
        return {k: self[k] for k in self}

    def __repr__(self):
        return repr(self.copy())


class SnakeVecEnv:
    def __init__(self, num_envs, num_snakes=4, device=None, seed=0, env_offset=0,
                 autoreset=True, coop=False, strict=False, lib_path=None, **env_kwargs):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError('SnakeVecEnv needs a HIP device (MI355X); there is no CPU fallback')
        self.num_envs = N = int(num_envs)
        self.cfg, self.meta = build_cfg(num_snakes=num_snakes, coop=coop, autoreset=autoreset,
                                        **env_kwargs)
        self.num_snakes = S = self.cfg.num_snakes
        self.autoreset = autoreset if autoreset == 'every_step' else bool(autoreset)
        self.strict = bool(strict)
        self.seed_base = int(seed) & 0xffffffff
        self.env_offset = int(env_offset)
        self._L = L = lib(lib_path)
        lay = SnakeLayout()
        check(L.snake_plan(ctypes.byref(self.cfg), N, ctypes.byref(lay)))
        self.layout = lay
        dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self._dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
        self.device = dev = torch.device('cuda', self._dev_index)
        self.obs_shape = (S, lay.obs_h, lay.obs_w, lay.obs_c)
        self.grid_shape = (self.cfg.height, self.cfg.width)
        self.action_n = 5 if self.cfg.observer == 1 else 3

        def buf(nbytes, dtype=torch.uint8):
            n = int(nbytes)
            return torch.zeros(max(n, 16), dtype=torch.uint8, device=dev)[:n].view(dtype)

        # state (layouts: include/snake_env.h snake_layout)
        self.grid = buf(lay.grid)
        self.snake = buf(lay.snake, torch.int32)
        self.body = buf(lay.body)
        self.env_rec = buf(lay.env, torch.int32)
        self.ctr = buf(lay.ctr, torch.int16)
        self.stats = buf(lay.stats, torch.float64)
        self.mt = buf(lay.mt, torch.int32)
        self.jscratch = buf(lay.jscratch, torch.int32) if lay.jscratch else None
        self.spawn = buf(lay.spawn, torch.int32)
        self.resetq = buf(lay.resetq, torch.int32)
        cap = int(lay.n_cand) * self.cfg.snake_length
        host = np.zeros(cap, np.int16)
        n = check(L.snake_build_candidates(ctypes.byref(self.cfg), host.ctypes.data_as(ctypes.c_void_p), cap))
        assert n == lay.n_cand
        self.cand = torch.from_numpy(host).to(dev)
        self._state = SnakeState(
            self.grid.data_ptr(), self.snake.data_ptr(), self.body.data_ptr(), self.env_rec.data_ptr(),
            self.ctr.data_ptr(), self.stats.data_ptr(), self.mt.data_ptr(), self.cand.data_ptr(),
            self.jscratch.data_ptr() if self.jscratch is not None else None,
            self.spawn.data_ptr(), self.resetq.data_ptr())
        with torch.cuda.device(dev):
            check(L.snake_seed(ctypes.byref(self.cfg), ctypes.byref(self._state), N, self.seed_base,
                               self.env_offset, self._stream()))

        self.single_action_space = spaces.Discrete(self.action_n)
        self.single_observation_space = spaces.Box(0, 255, self.obs_shape, np.uint8)
        self.observation_space = spaces.Box(0, 255, (N,) + self.obs_shape, np.uint8)
        self.action_space = spaces.Box(0, self.action_n - 1, (N, S), np.int64)
        self._reset_done = False
        self._palette = None
        self._plan_slab()
        # the step's ctypes call with its constant arguments prebuilt
        self._cfg_ref, self._state_ref = ctypes.byref(self.cfg), ctypes.byref(self._state)
        self._step_fn = L.snake_step

    # ------------------------------------------------------------------ utils
    def _stream(self):
        return ctypes.c_void_p(_raw_stream(self._dev_index))

    def sync(self):
        """Order the current stream after the background spawn-ahead kernel of
        the last step (include/snake_env.h snake_sync): call before reading or
        writing the state buffers directly. The methods here that touch state do."""
        torch = _torch()
        with torch.cuda.device(self.device):
            check(self._L.snake_sync(ctypes.byref(self.cfg), ctypes.byref(self._state), self.num_envs,
                                     self._stream()))

    # Outputs of one call (include/snake_env.h snake_out): the observations,
    # rewards and dones -- returned every step -- in fresh allocations of their
    # own (a buffer the caller drops is the one the next step gets back: an
    # allocation costs about as much as one view op, and a slab view of a typed
    # output takes three), the info outputs views of ONE fresh slab, made only
    # when read. Fresh per step (train_dqn.py:297 keeps references to returned
    # observations): four allocator calls instead of seven.
    # (name, dtype, per-env shape) in C-ABI order.
    _OUTS = ('obs', 'rew', 'done', 'ep_done', 'rank', 'ep_stats', 'err')
    _OWN = ('obs', 'rew', 'done')

    def _plan_slab(self):
        torch = _torch()
        N, S = self.num_envs, self.num_snakes
        spec = dict(obs=(torch.uint8, self.obs_shape), rew=(torch.float64, (S,)), done=(torch.bool, (S,)),
                    ep_done=(torch.bool, ()), rank=(torch.int32, (S,)), ep_stats=(torch.float64, (4, S)),
                    err=(torch.int32, ()))
        off, plan = 0, {}
        for k in self._OUTS:
            dt, shp = spec[k]
            n = N * int(np.prod(shp, dtype=np.int64)) * torch.empty((), dtype=dt).element_size()
            if k in self._OWN:
                plan[k] = (0, n, dt, (N,) + tuple(shp))
                continue
            plan[k] = (off, n, dt, (N,) + tuple(shp))
            off += (n + 255) // 256 * 256
        self._slab_plan, self._slab_bytes = plan, off
        self._obs_shape_n = (N,) + tuple(self.obs_shape)
        self._so = SnakeOut()

    def _new_out(self):
        """((obs, slab, rew, done), SnakeOut with their pointers); views via _view."""
        torch = _torch()
        dev, plan = self.device, self._slab_plan
        obs = torch.empty(self._obs_shape_n, dtype=torch.uint8, device=dev)
        rew = torch.empty(plan['rew'][3], dtype=torch.float64, device=dev)
        done = torch.empty(plan['done'][3], dtype=torch.bool, device=dev)
        slab = torch.empty(self._slab_bytes, dtype=torch.uint8, device=dev)
        base, so = slab.data_ptr(), self._so
        so.obs, so.rew, so.done = obs.data_ptr(), rew.data_ptr(), done.data_ptr()
        so.ep_done, so.rank, so.ep_stats, so.err = (base + plan[k][0] for k in self._OUTS[3:])
        return (obs, slab, rew, done), so

    _OWN_AT = {'obs': 0, 'rew': 2, 'done': 3}

    def _view(self, bufs, k):
        i = self._OWN_AT.get(k)
        if i is not None:
            return bufs[i]
        off, n, dt, shape = self._slab_plan[k]
        v = bufs[1][off:off + n]
        return (v if dt == _torch().uint8 else v.view(dt)).view(shape)

    def _actions(self, actions):
        torch = _torch()
        if (isinstance(actions, torch.Tensor) and actions.dtype == torch.int8 and actions.device == self.device
                and actions.is_contiguous() and actions.numel() == self.num_envs * self.num_snakes):
            return actions                          # the common case: device int8, used as is
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions))
        a = a.to(self.device)
        if a.dtype != torch.int8:
            if a.dtype.is_floating_point:
                bad = a != torch.floor(a)
                a = torch.where(bad, torch.full_like(a, -1), a)
            a = a.clamp(-128, 127).to(torch.int8)
        a = a.reshape(self.num_envs, self.num_snakes).contiguous()
        return a

    # ------------------------------------------------------------------- API
    def reset(self, mask=None):
        """SnakeEnv.reset (snake_env.py:131-159) for all envs, or those where mask is True.
        Returns the (N, S, h, w, 8*fs) uint8 observation tensor (rows of envs not in
        mask are left uninitialised)."""
        torch = _torch()
        slab, so = self._new_out()
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).reshape(self.num_envs).contiguous()
        with torch.cuda.device(self.device):
            check(self._L.snake_reset(ctypes.byref(self.cfg), ctypes.byref(self._state), self.num_envs,
                                      ctypes.c_void_p(m.data_ptr()) if m is not None else None,
                                      ctypes.byref(so), self._stream()))
        self._keep = m
        self._reset_done = True
        return self._view(slab, 'obs')

    def step(self, actions):
        """SnakeEnv.step (snake_env.py:301-414) for every env.

        actions: (N, S) ints ({0,1,2} for observer='snake', {0..4} for 'human').
        Returns (obs uint8 (N,S,h,w,C), rewards float64 (N,S), dones bool (N,S), info)
        with info tensors 'episode_done' (N,), 'rank' (N,S) and 'episode_scores',
        'episode_steps', 'episode_fruits', 'episode_kills' (N,S), meaningful where
        episode_done (zeros elsewhere); 'error' (N,) flags envs whose step was rejected
        for an invalid action (1: the reference's KeyError; such an env is left
        unchanged and reports reward 0 and done False) or whose auto-reset gave up
        finding disjoint spawn poses (2, see spawn_failures()).
        All outputs are freshly allocated every call."""
        if not self._reset_done:
            raise RuntimeError('call reset() before step()')
        a = self._actions(actions)
        slab, so = self._new_out()
        # (the library launches on the stream's own device whatever device is
        # current, snake_kernels.hip DeviceGuard; only the legacy null stream
        # takes the current device, so select ours for it)
        stream = _raw_stream(self._dev_index)
        if stream or _current_device() == self._dev_index:
            rc = self._step_fn(self._cfg_ref, self._state_ref, self.num_envs, a.data_ptr(), ctypes.byref(so), stream)
        else:
            with _torch().cuda.device(self.device):
                rc = self._step_fn(self._cfg_ref, self._state_ref, self.num_envs, a.data_ptr(), ctypes.byref(so),
                                   stream)
        if rc < 0:
            check(rc, self._L)
        self._keep = a
        info = _StepInfo(self, slab, stream)
        if self.strict and bool(info['error'].any()):
            err = info['error']
            bad = (err == 1).nonzero().flatten().tolist()
            if bad:
                raise KeyError(f'invalid action for an alive snake in envs {bad[:8]}')
            raise RuntimeError(f'auto-reset gave up placing disjoint snakes in envs '
                               f'{(err == 2).nonzero().flatten().tolist()[:8]}')
        return slab[0], slab[2], slab[3], info

    def render_rgb(self):
        """rgb_from_grid of every env's current grid (grid_util.py:164-175), on the
        device: (N, H, W, 3) uint8, freshly allocated (kernel k_render)."""
        torch = _torch()
        H, W = self.grid_shape
        rgb = torch.empty((self.num_envs, H, W, 3), dtype=torch.uint8, device=self.device)
        if self._palette is None:
            from .core.render import palette
            self._palette = np.ascontiguousarray(palette())
        with torch.cuda.device(self.device):
            check(self._L.snake_render_rgb(ctypes.byref(self.cfg), ctypes.byref(self._state), self.num_envs,
                                           self._palette.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_void_p(rgb.data_ptr()), self._stream()))
        return rgb

    # --------------------------------------------------------- introspection
    def grids(self):
        """Current grid of every env, (N, H, W) uint8 cell values 10*idx + code
        (newest ring slot)."""
        torch = _torch()
        lay, fs = self.layout, self.cfg.frame_stack
        H, W = self.grid_shape
        ring = self.grid.view(self.num_envs, fs, lay.grid_stride)
        cur = self.env_rec.view(self.num_envs, 8)[:, 2].long()
        g = ring[torch.arange(self.num_envs, device=self.device), cur][:, :H * W]
        return g.reshape(self.num_envs, H, W)

    def spawn_failures(self):
        """(N,) int32: 1 where the env's last reset gave up after 2^16 spawn
        permutations without S disjoint poses (its snakes may overlap). snake_plan
        rejects boards where that is likelier than ~2e-6 per reset."""
        return self.env_rec.view(self.num_envs, 8)[:, 5]

    # ------------------------------------------------------- snapshot/restore
    # The spawn-ahead records (snake_layout.spawn) and the status word that points
    # at them (env word 4: status, record buffer, generation) are a cache of
    # draws the next reset would make anyway (include/snake_env.h snake_step).
    # With the background spawn kernel, which envs hold a record at a given
    # moment depends on when each k_spawn ran, so snapshots hold the env state
    # without the cache: word 4 in its canonical form 0 (no record; the next
    # reset of the env draws from its MT19937 state, with identical results).
    _STATE_BUFFERS = ('grid', 'snake', 'body', 'env_rec', 'ctr', 'stats', 'mt')

    def env_records(self):
        """(N, 8) int32 copy of the env records (alive_snakes, episode_length, ring
        slot, MT position, spawn-ahead status, give-up flag, 0, 0) with word 4 in
        its canonical form (0: no spawn-ahead record), ordered after the
        background spawn kernel. Deterministic for any spawn-ahead mode, timing
        and shard split."""
        self.sync()
        er = self.env_rec.view(self.num_envs, 8).clone()
        er[:, 4] = 0
        return er

    def state_dict(self, device=None):
        """Snapshot of the whole batch: the persistent env state of snake_layout
        (grid ring, snake records, body rings, env records, crop centres, episode
        statistics, MT19937 keys) copied (to `device`, default: this env's device)
        plus the configuration it belongs to. The spawn-ahead cache is not saved
        (env word 4 canonical, env_records()), and the step's queues and link
        tables are transient (empty between steps): two snapshots of the same env
        state are equal whatever the spawn-ahead mode or timing. load_state_dict()
        on this or a fresh SnakeVecEnv of the same configuration continues
        bit-identically; the tensors can be torch.save()d beside a learner
        checkpoint (train_dqn.py:356-383)."""
        torch = _torch()
        dev = torch.device(device) if device is not None else self.device
        self.sync()
        sd = {k: getattr(self, k).detach().to(dev, copy=True) for k in self._STATE_BUFFERS if k != 'env_rec'}
        sd['env_rec'] = self.env_records().view(-1).to(dev)
        torch.cuda.current_stream(self.device).synchronize()
        sd['meta'] = self._snapshot_meta()
        return sd

    def _snapshot_meta(self):
        lay = self.layout
        return dict(abi=int(self._L.snake_abi_version()), num_envs=self.num_envs,
                    cfg=[getattr(self.cfg, f) for f, _ in self.cfg._fields_
                         if f not in ('spawn_ahead', 'spawn_background')],
                    sizes=[int(getattr(lay, k)) for k in ('grid', 'snake', 'body', 'env', 'ctr', 'stats', 'mt')],
                    seed=self.seed_base, env_offset=self.env_offset, reset_done=self._reset_done)

    def load_state_dict(self, sd):
        """Restore a state_dict() snapshot (same configuration and num_envs,
        checked); the next step continues exactly where the snapshot was taken
        (the spawn-ahead records are drawn afresh: env word 4 is 0)."""
        torch = _torch()
        mine, theirs = self._snapshot_meta(), sd['meta']
        for key in ('abi', 'num_envs', 'cfg', 'sizes'):
            if mine[key] != theirs[key]:
                raise ValueError(f'snapshot does not match this env: {key} {theirs[key]} != {mine[key]}')
        self.sync()
        with torch.cuda.device(self.device):
            for k in self._STATE_BUFFERS:
                getattr(self, k).copy_(sd[k].to(self.device))
            self.env_rec.view(self.num_envs, 8)[:, 4] = 0
        self.seed_base, self.env_offset = theirs['seed'], theirs['env_offset']
        self._reset_done = bool(theirs['reset_done'])

    def alive_counters(self):
        return self.env_rec.view(self.num_envs, 8)[:, 0]

    def episode_lengths(self):
        return self.env_rec.view(self.num_envs, 8)[:, 1]

    def snake_table(self):
        """(N, S, 7) int32: head r,c, tail r,c, dir (0 UP,1 RIGHT,2 DOWN,3 LEFT), alive, length."""
        torch = _torch()
        r = self.snake.view(self.num_envs, self.num_snakes, 4)
        x, y, z = r[..., 0], r[..., 1], r[..., 2]
        return torch.stack([x & 255, (x >> 8) & 255, (x >> 16) & 255, (x >> 24) & 255,
                            y & 3, (y >> 8) & 1, ((z >> 16) & 0xffff) + 1], dim=-1)

    def mt_state(self):
        """(N, 624) MT19937 keys (int32 view of uint32) and (N,) positions (read-only
        use: writers go through set_mt_state). A position above 624 means the key's
        twist is pending: position 624 + j is word j of the next key (numpy's
        state is the twisted key at position - 624)."""
        return self.mt.view(self.num_envs, 624), self.env_rec.view(self.num_envs, 8)[:, 3]

    def set_mt_state(self, i, key, pos):
        """Overwrite env i's MT19937 key (624 uint32, as int32) and position; voids
        its spawn-ahead record (include/snake_env.h), which was drawn from the old state."""
        torch = _torch()
        self.sync()
        er = self.env_rec.view(self.num_envs, 8)
        self.mt.view(self.num_envs, 624)[i].copy_(torch.as_tensor(key).to(self.device))
        er[i, 3] = int(pos)
        er[i, 4] = 0

    def inject(self, i, grid, snakes, alive_snakes, episode_length=0):
        """Overwrite env i with a crafted state (the env.grid / env.snakes assignment
        the reference allows): grid (H, W) cell values, snakes = [(coords, alive)]
        with coords [(r, c), ...] head first (core/snake.py:53-74). The frame
        stack is refilled with this grid and the episode statistics are zeroed, as
        _init_obs/_reset_epi_stats do; the env's MT19937 stream is left as is."""
        torch = _torch()
        self.sync()
        H, W = self.grid_shape
        S, fs, lay = self.num_snakes, self.cfg.frame_stack, self.layout
        g = np.zeros(lay.grid_stride, np.uint8)
        g[:H * W] = np.asarray(grid, np.int64).reshape(-1).astype(np.uint8)
        ring = torch.from_numpy(np.tile(g, fs)).to(self.device)
        self.grid.view(self.num_envs, fs * lay.grid_stride)[i].copy_(ring)
        rec = np.zeros((S, 4), np.int32)
        body = np.zeros((S, lay.ring_cap), np.uint8)
        dmap = {(-1, 0): 0, (0, 1): 1, (1, 0): 2, (0, -1): 3}
        for k, (coords, alive) in enumerate(snakes):
            co = [tuple(int(x) for x in c) for c in coords]
            dirs = [dmap[(a[0] - b[0], a[1] - b[1])] for a, b in zip(co[:-1], co[1:])]
            body[k, :len(dirs)] = dirs
            (hr, hc), (tr, tc) = co[0], co[-1]
            x = hr | (hc << 8) | (tr << 16) | (tc << 24)
            # rec.w: the tail queue (directions[-1], count 1), see k_logic
            rec[k] = [x - (1 << 32) if x >= (1 << 31) else x, dirs[0] | (int(bool(alive)) << 8),
                      (len(co) - 1) << 16, dirs[-1] | (1 << 28)]
        # crop centres of the refilled frames: the own HEAD cell (argmax of the own
        # head plane, snake_env.py:500-501), (0, 0) when there is none
        g2 = np.asarray(grid, np.int64).reshape(H, W)
        ctr = np.zeros(S, np.int16)
        for k in range(S):
            hits = np.argwhere(g2 == 3 + 10 * k)
            if len(hits):
                ctr[k] = (int(hits[0][0]) << 8) | int(hits[0][1])
        self.ctr.view(self.num_envs, fs * S)[i].copy_(torch.from_numpy(np.tile(ctr, fs)).to(self.device))
        self.snake.view(self.num_envs, S * 4)[i].copy_(torch.from_numpy(rec.reshape(-1)).to(self.device))
        self.body.view(self.num_envs, S * lay.ring_cap)[i].copy_(torch.from_numpy(body.reshape(-1)).to(self.device))
        er = self.env_rec.view(self.num_envs, 8)
        er[i, 0] = int(alive_snakes)
        er[i, 1] = int(episode_length)
        er[i, 2] = fs - 1
        self.stats.view(self.num_envs, -1)[i].zero_()
        self._reset_done = True

    def close(self):
        # the state buffers go back to the allocator on the current stream: order
        # that after a background spawn kernel still writing them, then release
        # the library's background streams and events for this state (snake_release)
        if getattr(self, '_state', None) is not None and torch_cuda_alive():
            try:
                self.sync()
                self._L.snake_release(ctypes.byref(self.cfg), ctypes.byref(self._state), self.num_envs)
            except Exception:
                pass
            self._state = None

    def __del__(self):
        self.close()
