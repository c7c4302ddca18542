"""ctypes binding of libsnake_amd.so (C-ABI declared in include/snake_env.h).

The product has no CPU fallback: if the HIP library is missing or fails to
load, every env constructor raises. Build it with ``python __graft_entry__.py``
(or ``make -C marl-snake_amd/csrc``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libsnake_amd.so')

SNAKE_ABI_VERSION = 17

# Symbols include/snake_env.h declares (checked by tests/test_capi.py).
EXPORTS = ('snake_plan', 'snake_build_candidates', 'snake_seed', 'snake_reset', 'snake_step',
           'snake_sync', 'snake_release', 'snake_render_rgb', 'snake_timing_enable', 'snake_timing_read', 'snake_debug_set', 'snake_last_error', 'snake_abi_version',
           'snake_dqn_plan', 'snake_dqn_rows', 'snake_dqn_forward', 'snake_dqn32_scratch', 'snake_dqn32_forward')


class SnakeCfg(ctypes.Structure):
    _fields_ = [('height', ctypes.c_int32), ('width', ctypes.c_int32),
                ('num_snakes', ctypes.c_int32), ('snake_length', ctypes.c_int32),
                ('vision_range', ctypes.c_int32), ('frame_stack', ctypes.c_int32),
                ('observer', ctypes.c_int32), ('num_fruits', ctypes.c_int32),
                ('rew_fruit', ctypes.c_double), ('rew_kill', ctypes.c_double),
                ('rew_lose', ctypes.c_double), ('rew_win', ctypes.c_double),
                ('rew_time', ctypes.c_double), ('max_episode_steps', ctypes.c_double),
                ('coop', ctypes.c_int32), ('autoreset', ctypes.c_int32), ('spawn_ahead', ctypes.c_int32),
                ('spawn_background', ctypes.c_int32)]


class SnakeLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        'grid', 'snake', 'body', 'env', 'ctr', 'stats', 'mt', 'cand', 'jscratch', 'spawn', 'resetq',
        'obs', 'rew',
        'done',
        'ep_done', 'rank', 'ep_stats', 'err', 'n_cand')] + [
        ('obs_h', ctypes.c_int32), ('obs_w', ctypes.c_int32), ('obs_c', ctypes.c_int32),
        ('grid_stride', ctypes.c_int32), ('ring_cap', ctypes.c_int32)]


class SnakeState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        'grid', 'snake', 'body', 'env', 'ctr', 'stats', 'mt', 'cand', 'jscratch', 'spawn', 'resetq')]


class SnakeOut(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        'obs', 'rew', 'done', 'ep_done', 'rank', 'ep_stats', 'err')]


class DqnCfg(ctypes.Structure):
    _fields_ = [('height', ctypes.c_int32), ('width', ctypes.c_int32), ('channels', ctypes.c_int32),
                ('num_actions', ctypes.c_int32), ('conv_waves', ctypes.c_int32)]


class DqnLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ('conv1_w', 'conv2_w', 'conv3_w', 'fc1_w', 'fc2_w', 'act_per_obs')] + [
        (n, ctypes.c_int32) for n in ('cpad', 'p16', 'k1', 'lds_conv')]


class DqnNet(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        'conv1_w', 'conv2_w', 'conv3_w', 'fc1_w', 'fc2_w', 'conv1_b', 'conv2_b', 'conv3_b', 'fc1_b', 'fc2_b',
        'fc3_w', 'fc3_b')]


class Dqn32Net(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        'conv1_w', 'conv2_w', 'conv3_w', 'fc1_w', 'fc2_w', 'fc3_w', 'conv1_b', 'conv2_b', 'conv3_b', 'fc1_b',
        'fc2_b', 'fc3_b')]


class NativeError(RuntimeError):
    pass


_libs = {}


def lib(path=None):
    """Load libsnake_amd.so once; raise loudly when it is absent. `path` loads an
    alternative build of the same ABI (A/B timing of kernel variants)."""
    path = path or os.environ.get("SNAKE_LIB") or LIB_PATH
    if path in _libs:
        return _libs[path]
    # PyTorch owns device memory and streams: its HIP runtime must be the one in
    # the process before libsnake_amd.so resolves libamdhip64.so.7 (loading ours
    # first brings in /opt/rocm's copy beside torch's, and launches then fail
    # with "no ROCm-capable device").
    import torch  # noqa: F401
    if not os.path.exists(path):
        raise NativeError(f'{path} not built: run `python __graft_entry__.py` '
                          '(hipcc --offload-arch=gfx950); there is no CPU fallback')
    L = ctypes.CDLL(path)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    L.snake_abi_version.restype = ctypes.c_int
    L.snake_last_error.restype = ctypes.c_char_p
    L.snake_plan.argtypes = [ctypes.POINTER(SnakeCfg), I64, ctypes.POINTER(SnakeLayout)]
    L.snake_build_candidates.restype = I64
    L.snake_build_candidates.argtypes = [ctypes.POINTER(SnakeCfg), P, I64]
    L.snake_seed.argtypes = [ctypes.POINTER(SnakeCfg), ctypes.POINTER(SnakeState), I64,
                             ctypes.c_uint32, I64, P]
    L.snake_reset.argtypes = [ctypes.POINTER(SnakeCfg), ctypes.POINTER(SnakeState), I64, P,
                              ctypes.POINTER(SnakeOut), P]
    L.snake_step.argtypes = [ctypes.POINTER(SnakeCfg), ctypes.POINTER(SnakeState), I64, P,
                             ctypes.POINTER(SnakeOut), P]
    L.snake_sync.argtypes = [ctypes.POINTER(SnakeCfg), ctypes.POINTER(SnakeState), I64, P]
    L.snake_release.argtypes = [ctypes.POINTER(SnakeCfg), ctypes.POINTER(SnakeState), I64]
    L.snake_render_rgb.argtypes = [ctypes.POINTER(SnakeCfg), ctypes.POINTER(SnakeState), I64, P, P, P]
    L.snake_dqn_plan.argtypes = [ctypes.POINTER(DqnCfg), ctypes.POINTER(DqnLayout)]
    L.snake_dqn_rows.argtypes = [ctypes.POINTER(DqnCfg), P, I64]
    L.snake_dqn_rows.restype = I64
    L.snake_dqn_forward.argtypes = [ctypes.POINTER(DqnCfg), ctypes.POINTER(DqnNet), P, I64, P, P, P, P]
    L.snake_dqn32_scratch.argtypes = [ctypes.POINTER(DqnCfg), I64]
    L.snake_dqn32_scratch.restype = I64
    L.snake_dqn32_forward.argtypes = [ctypes.POINTER(DqnCfg), ctypes.POINTER(Dqn32Net), P, I64, P, P, P, P]
    L.snake_timing_enable.argtypes = [ctypes.c_int]
    L.snake_debug_set.argtypes = [ctypes.c_char_p, ctypes.c_longlong]
    L.snake_timing_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_int64)]
    if L.snake_abi_version() != SNAKE_ABI_VERSION:
        raise NativeError('libsnake_amd.so ABI version mismatch; rebuild it')
    _libs[path] = L
    return L


def timing_enable(on, L=None):
    check((L or lib()).snake_timing_enable(1 if on else 0), L)


def debug_set(name, value, L=None):
    """snake_debug_set (include/snake_env.h): a process-wide testing knob."""
    check((L or lib()).snake_debug_set(name.encode(), int(value)), L)


def timing_read(kernel, L=None):
    """(total device ms, launches) of one kernel since its last read; for
    kernel='resets' / 'resets_timed' / 'spawn_hits' / 'spawn_jobs' a count (ms is 0)."""
    L = L or lib()
    ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
    check(L.snake_timing_read(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)), L)
    return ms.value, n.value


def check(rc, L=None):
    if rc < 0:
        msg = (L or lib()).snake_last_error().decode(errors='replace')
        if rc == -1:
            raise ValueError(msg)
        raise NativeError(f'snake C-ABI error {rc}: {msg}')
    return rc
