"""Fused consumer of the observations: the reference's DQN forward on the GPU.

The reference trains a shared DQN on the env's observations (train_dqn.py:104-151;
the same network is the frozen feature extractor of train_ga.py:60-100):

    x = obs.permute(0, 3, 1, 2).float()        # NHWC uint8 -> NCHW (0/1 values)
    x = relu(conv1(x)); x = relu(conv2(x)); x = relu(conv3(x))   # 3x3, pad 1
    x = relu(fc1(x.reshape(B, -1))); x = relu(fc2(x))            # forward_features
    q = fc3(x)

DQNForward runs it through snake_dqn_forward (marl-snake_amd/csrc/dqn_kernels.hip):
implicit-GEMM convolutions and the fc layers on the bf16 matrix cores, fp32
accumulation. The weights come from a state dict with the reference's parameter
names (conv1.weight, ..., fc3.bias) and are packed once into the kernel layouts
(include/snake_env.h snake_dqn_layout); packing is a layout transform done with
torch ops, the forward pass is the HIP kernels only.
"""
import ctypes

from ._native import Dqn32Net, DqnCfg, DqnLayout, DqnNet, check, lib


def _torch():
    import torch
    return torch


# The reference network's parameter shapes (train_dqn.py:104-151): the kernels
# hard-code 32/64/64 conv channels and 256/128 fc widths, so a mismatched state
# dict must raise here instead of making them read past the packed weights.
def _check_shapes(state, C, P, A):
    want = {'conv1.weight': (32, C, 3, 3), 'conv1.bias': (32,),
            'conv2.weight': (64, 32, 3, 3), 'conv2.bias': (64,),
            'conv3.weight': (64, 64, 3, 3), 'conv3.bias': (64,),
            'fc1.weight': (256, 64 * P), 'fc1.bias': (256,),
            'fc2.weight': (128, 256), 'fc2.bias': (128,),
            'fc3.weight': (A, 128), 'fc3.bias': (A,)}
    for name, shape in want.items():
        if name not in state:
            raise ValueError('state dict has no %s' % name)
        got = tuple(state[name].shape)
        if got != shape:
            raise ValueError('%s shape %s != %s' % (name, got, shape))


class DQNForward:
    """DQN(input_shape=(N, h, w, c), num_actions) forward on uint8 NHWC observations.

    state: a state dict (or nn.Module) of the reference DQN (conv1..conv3, fc1..fc3).
    conv_waves: waves per observation in the conv kernel (0 = the library default).
    precision: 'bf16' (the fused MFMA kernels: bf16 products, fp32 accumulation;
    square odd maps up to 11x11, 8-32 channels) or 'fp32' (dqn32_kernels.hip:
    fp32 arithmetic on any map, e.g. train_dqn.py's 20x20 full-map Config)."""

    def __init__(self, state, height, width, channels, num_actions=3, device=None, lib_path=None, conv_waves=0,
                 precision='bf16'):
        torch = _torch()
        if hasattr(state, 'state_dict'):
            state = state.state_dict()
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self._L = L = lib(lib_path)
        self.cfg = DqnCfg(int(height), int(width), int(channels), int(num_actions), int(conv_waves))
        if precision not in ('bf16', 'fp32'):
            raise ValueError("precision must be 'bf16' or 'fp32'")
        self.precision = precision
        self.num_actions = int(num_actions)
        self._scratch = None
        _check_shapes(state, int(channels), int(height) * int(width), int(num_actions))
        if precision == 'fp32':
            self._init_fp32(state)
            return
        lay = DqnLayout()
        check(L.snake_dqn_plan(ctypes.byref(self.cfg), ctypes.byref(lay)), L)
        self.layout = lay
        H, W, C, A = int(height), int(width), int(channels), int(num_actions)
        P, P16, CP, K1 = H * W, lay.p16, lay.cpad, lay.k1
        d = self.device
        f32 = dict(dtype=torch.float32, device=d)

        def g(name):
            return state[name].detach().to(**f32)

        def bits(t):          # bf16 bit patterns as int16 (the kernels' uint16 words)
            return t.to(torch.bfloat16).contiguous().view(torch.int16)

        def conv_pack(w, cin_pad, k_pad):
            # [out][in][ky][kx] -> B[out][k = (ky*3 + kx) * cin_pad + ci], zero padded,
            # stored in MFMA fragment order: [out/16][k/32][k%32 / 8][out%16][8]
            out_ch, cin = w.shape[0], w.shape[1]
            t = torch.zeros((out_ch, 9, cin_pad), **f32)
            t[:, :, :cin] = w.permute(0, 2, 3, 1).reshape(out_ch, 9, cin)
            flat = torch.zeros((out_ch, k_pad), **f32)
            flat[:, :9 * cin_pad] = t.reshape(out_ch, 9 * cin_pad)
            frag = flat.reshape(out_ch // 16, 16, k_pad // 32, 4, 8).permute(0, 2, 3, 1, 4)
            return bits(frag.contiguous().reshape(out_ch, k_pad))

        w1, w2, w3 = g('conv1.weight'), g('conv2.weight'), g('conv3.weight')
        if tuple(w1.shape) != (32, C, 3, 3) or tuple(w2.shape) != (64, 32, 3, 3) or tuple(w3.shape) != (64, 64, 3, 3):
            raise ValueError('state dict does not match DQN(input_shape=(.., %d, %d, %d))' % (H, W, C))
        fc1 = g('fc1.weight')
        if tuple(fc1.shape) != (256, 64 * P):
            raise ValueError('fc1.weight shape %s != (256, %d)' % (tuple(fc1.shape), 64 * P))
        # k in conv3's fragment order (snake_env.h snake_dqn_layout.fc1_w) -> the
        # reference's NCHW flatten index channel * h*w + position
        rows = (ctypes.c_int32 * P16)()
        n = L.snake_dqn_rows(ctypes.byref(self.cfg), ctypes.cast(rows, ctypes.c_void_p), P16)
        if n != P16:
            check(int(n) if n < 0 else -1, L)
        rowpos = torch.tensor(list(rows), dtype=torch.int64, device=d)
        k = torch.arange(64 * P16, device=d)
        r, j, c16, quad = k % 4, (k // 4) % 2, (k // 8) % 16, (k // 128) % 4
        half, m = (k // 512) % 2, k // 1024
        ch, p = (2 * half + j) * 16 + c16, rowpos[m * 16 + 4 * quad + r]
        src = torch.where(p >= 0, ch * P + p, 0)
        fc1p = torch.where((p >= 0)[None, :], fc1[:, src], torch.zeros((), **f32))
        fc3 = g('fc3.weight')
        if tuple(fc3.shape) != (A, 128):
            raise ValueError('fc3.weight shape %s != (%d, 128)' % (tuple(fc3.shape), A))
        self.tensors = dict(
            conv1_w=conv_pack(w1, CP, K1), conv2_w=conv_pack(w2, 32, 288), conv3_w=conv_pack(w3, 64, 576),
            fc1_w=bits(fc1p), fc2_w=bits(g('fc2.weight')),
            conv1_b=g('conv1.bias'), conv2_b=g('conv2.bias'), conv3_b=g('conv3.bias'),
            fc1_b=g('fc1.bias'), fc2_b=g('fc2.bias'), fc3_w=fc3.contiguous(), fc3_b=g('fc3.bias'))
        for k, n in (('conv1_w', lay.conv1_w), ('conv2_w', lay.conv2_w), ('conv3_w', lay.conv3_w),
                     ('fc1_w', lay.fc1_w), ('fc2_w', lay.fc2_w)):
            assert self.tensors[k].numel() == n, (k, self.tensors[k].numel(), n)
        self.net = DqnNet(*(self.tensors[k].data_ptr() for k in (
            'conv1_w', 'conv2_w', 'conv3_w', 'fc1_w', 'fc2_w', 'conv1_b', 'conv2_b', 'conv3_b', 'fc1_b',
            'fc2_b', 'fc3_w', 'fc3_b')))
        self.num_actions = A
        self._scratch = None

    def _init_fp32(self, state):
        """fp32 weights, row-major [out][in] (include/snake_env.h snake_dqn32_net);
        fc1's columns permuted from the NCHW flatten to NHWC."""
        torch = _torch()
        H, W, C, A = self.cfg.height, self.cfg.width, self.cfg.channels, self.cfg.num_actions
        P = H * W
        n = self._L.snake_dqn32_scratch(ctypes.byref(self.cfg), 0)
        check(int(n) if n < 0 else 0, self._L)
        f32 = dict(dtype=torch.float32, device=self.device)

        def g(name):
            return state[name].detach().to(**f32)

        def conv(w, cin):
            if tuple(w.shape[1:]) != (cin, 3, 3):
                raise ValueError('conv weight shape %s does not match %d input channels' % (tuple(w.shape), cin))
            return w.permute(0, 2, 3, 1).reshape(w.shape[0], 9 * cin).contiguous()
        fc1 = g('fc1.weight')
        if tuple(fc1.shape) != (256, 64 * P):
            raise ValueError('fc1.weight shape %s != (256, %d)' % (tuple(fc1.shape), 64 * P))
        fc3 = g('fc3.weight')
        if tuple(fc3.shape) != (A, 128):
            raise ValueError('fc3.weight shape %s != (%d, 128)' % (tuple(fc3.shape), A))
        self.tensors = dict(
            conv1_w=conv(g('conv1.weight'), C), conv2_w=conv(g('conv2.weight'), 32),
            conv3_w=conv(g('conv3.weight'), 64),
            fc1_w=fc1.reshape(256, 64, P).permute(0, 2, 1).reshape(256, P * 64).contiguous(),
            fc2_w=g('fc2.weight').contiguous(), fc3_w=fc3.contiguous(),
            conv1_b=g('conv1.bias'), conv2_b=g('conv2.bias'), conv3_b=g('conv3.bias'),
            fc1_b=g('fc1.bias'), fc2_b=g('fc2.bias'), fc3_b=g('fc3.bias'))
        self.net = Dqn32Net(*(self.tensors[k].data_ptr() for k in (
            'conv1_w', 'conv2_w', 'conv3_w', 'fc1_w', 'fc2_w', 'fc3_w', 'conv1_b', 'conv2_b', 'conv3_b',
            'fc1_b', 'fc2_b', 'fc3_b')))

    def _run(self, obs, features):
        torch = _torch()
        H, W, C = self.cfg.height, self.cfg.width, self.cfg.channels
        if obs.dim() == 3:
            obs = obs.unsqueeze(0)
        obs = obs.reshape(-1, H, W, C)
        if obs.dtype != torch.uint8:
            raise TypeError('DQNForward takes the env observations as uint8 (got %s)' % obs.dtype)
        obs = obs.to(self.device).contiguous()
        B = obs.shape[0]
        if self.precision == 'fp32':
            return self._run32(obs, B, features)
        need = B * self.layout.act_per_obs
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.int16, device=self.device)
        q = torch.empty((B, self.num_actions), dtype=torch.float32, device=self.device)
        feat = torch.empty((B, 128), dtype=torch.float32, device=self.device) if features else None
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check(self._L.snake_dqn_forward(ctypes.byref(self.cfg), ctypes.byref(self.net),
                                        ctypes.c_void_p(obs.data_ptr()), B,
                                        ctypes.c_void_p(self._scratch.data_ptr()),
                                        ctypes.c_void_p(q.data_ptr()),
                                        ctypes.c_void_p(feat.data_ptr()) if features else None, stream), self._L)
        self._keep = obs
        return q, feat

    def _run32(self, obs, B, features):
        torch = _torch()
        need = int(self._L.snake_dqn32_scratch(ctypes.byref(self.cfg), B))
        check(need if need < 0 else 0, self._L)
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
        q = torch.empty((B, self.num_actions), dtype=torch.float32, device=self.device)
        feat = torch.empty((B, 128), dtype=torch.float32, device=self.device) if features else None
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check(self._L.snake_dqn32_forward(ctypes.byref(self.cfg), ctypes.byref(self.net),
                                          ctypes.c_void_p(obs.data_ptr()), B,
                                          ctypes.c_void_p(self._scratch.data_ptr()),
                                          ctypes.c_void_p(q.data_ptr()),
                                          ctypes.c_void_p(feat.data_ptr()) if features else None, stream), self._L)
        self._keep = obs
        return q, feat

    def __call__(self, obs):
        """DQN.forward: (B, h, w, c) uint8 -> (B, A) float32 Q-values."""
        return self._run(obs, False)[0]

    def forward_features(self, obs):
        """DQN.forward_features: (B, h, w, c) uint8 -> (B, 128) float32 (relu(fc2))."""
        return self._run(obs, True)[1]
