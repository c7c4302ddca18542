"""The fused DQN consumer (marl-snake_amd/csrc/dqn_kernels.hip) against a plain
PyTorch fp32 restatement of the reference network (train_dqn.py:104-151).

fp32 mode (precision='fp32', dqn32_kernels.hip): fp32 arithmetic on any map
(train_dqn.py's 20x20 full-map Config included); held to |err| <= 1e-5 * max|ref|
against a float64 CPU restatement (no reduced-precision conv/matmul paths).

Tolerance (bf16 mode): the matrix products take bf16 inputs (weights and activations are
rounded to bf16 between layers, 8 significant bits) with fp32 accumulation, so
outputs agree with the fp32 reference to |err| <= 2e-2 * max|ref| + 1e-3 (a
bf16-emulating reference agrees to <= 2e-3 * max|ref|, which pins the layouts)."""
import pytest

torch = pytest.importorskip('torch')
nn = torch.nn
F = torch.nn.functional


class RefDQN(nn.Module):
    """train_dqn.py:104-151, restated (layers, flatten order, ReLUs)."""

    def __init__(self, h, w, c, num_actions):
        super().__init__()
        self.conv1 = nn.Conv2d(c, 32, kernel_size=3, stride=1, padding=1)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=3, stride=1, padding=1)
        self.conv3 = nn.Conv2d(64, 64, kernel_size=3, stride=1, padding=1)
        self.fc1 = nn.Linear(h * w * 64, 256)
        self.fc2 = nn.Linear(256, 128)
        self.fc3 = nn.Linear(128, num_actions)

    def forward_features(self, x, bf16=False):
        r = (lambda t: t.to(torch.bfloat16).float()) if bf16 else (lambda t: t)
        x = x.permute(0, 3, 1, 2).to(self.conv1.weight.dtype)   # .float() (float64 for the fp32-mode check)
        x = x / 255.0 if x.max() > 1.0 else x
        def lin(layer, t):
            return F.linear(r(t), r(layer.weight), layer.bias)
        def conv(layer, t):
            return F.conv2d(r(t), r(layer.weight), layer.bias, padding=1)
        x = F.relu(conv(self.conv1, x))
        x = F.relu(conv(self.conv2, x))
        x = F.relu(conv(self.conv3, x))
        x = x.reshape(x.size(0), -1)
        x = F.relu(lin(self.fc1, x))
        return F.relu(lin(self.fc2, x))

    def forward(self, x, bf16=False):
        return F.linear(self.forward_features(x, bf16), self.fc3.weight, self.fc3.bias)


def test_dqn_plan_sizes():
    import ctypes
    from marlenv import _native
    lay = _native.DqnLayout()
    cfg = _native.DqnCfg(11, 11, 8, 3)
    assert _native.lib().snake_dqn_plan(ctypes.byref(cfg), ctypes.byref(lay)) == 0
    assert (lay.cpad, lay.p16, lay.k1) == (8, 128, 96)
    assert lay.fc1_w == 256 * 64 * 128 and lay.act_per_obs == 64 * 128
    bad = _native.DqnCfg(20, 20, 8, 3)           # full 20x20 map: vision_range <= 5 only
    assert _native.lib().snake_dqn_plan(ctypes.byref(bad), ctypes.byref(lay)) == -1
    for vr in range(1, 6):      # GEMM rows cover every position once; a tile's border cells differ mod 16
        W = 2 * vr + 1
        c = _native.DqnCfg(W, W, 8, 3)
        n = _native.lib().snake_dqn_rows(ctypes.byref(c), None, 0)
        rows = (ctypes.c_int32 * n)()
        assert _native.lib().snake_dqn_rows(ctypes.byref(c), ctypes.cast(rows, ctypes.c_void_p), n) == n
        rows = list(rows)
        assert sorted(x for x in rows if x >= 0) == list(range(W * W))
        for t in range(n // 16):
            q = [((p // W + 1) * (W + 2) + p % W + 1) % 16 for p in rows[16 * t:16 * t + 16] if p >= 0]
            assert len(set(q)) == len(q)
    for h, w, c, a, nw in ((11, 9, 8, 3, 0), (11, 11, 12, 3, 0), (11, 11, 40, 3, 0), (11, 11, 8, 5, 0),
                           (4, 4, 8, 3, 0), (11, 11, 8, 3, 3)):
        assert _native.lib().snake_dqn_plan(ctypes.byref(_native.DqnCfg(h, w, c, a, nw)), ctypes.byref(lay)) == -1


def _obs_batch(B, vr, fs, S=4, seed=0):
    """Real observations: a short random rollout of the GPU env."""
    from marlenv import SnakeVecEnv
    n = max(1, -(-B // S))
    v = SnakeVecEnv(n, num_snakes=S, seed=seed, height=20, width=20, vision_range=vr, frame_stack=fs)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(seed)
    for _ in range(12):
        o, _, _, _ = v.step(torch.randint(0, 3, (n, S), generator=g, device='cuda', dtype=torch.int8))
    return o.reshape(-1, *o.shape[2:])[:B].contiguous()


@pytest.mark.gpu
@pytest.mark.parametrize('B,vr,fs,waves', [(512, 5, 1, 0), (333, 5, 1, 0), (64, 4, 2, 0), (40, 3, 4, 0),
                                           (1, 5, 1, 0), (257, 2, 1, 0), (100, 1, 3, 0), (3000, 5, 2, 0),
                                           (333, 5, 1, 1), (333, 5, 1, 2), (64, 4, 2, 1), (257, 2, 1, 4)])
def test_dqn_forward_matches_fp32_reference(B, vr, fs, waves):
    from marlenv.dqn import DQNForward
    torch.manual_seed(1)
    h = w = 2 * vr + 1
    c = 8 * fs
    ref = RefDQN(h, w, c, 3).cuda()
    obs = _obs_batch(B, vr, fs)
    assert obs.shape == (B, h, w, c)
    net = DQNForward(ref, h, w, c, 3, conv_waves=waves)
    q = net(obs)
    feat = net.forward_features(obs)
    torch.cuda.synchronize()
    with torch.no_grad():
        q32 = ref(obs)
        f32 = ref.forward_features(obs)
        qbf = ref(obs, bf16=True)
    assert q.shape == (B, 3) and feat.shape == (B, 128)
    assert torch.isfinite(q).all()
    scale = float(q32.abs().max())
    assert float((q - q32).abs().max()) <= 2e-2 * scale + 1e-3
    assert float((q - qbf).abs().max()) <= 2e-3 * scale + 1e-4
    fs_ = float(f32.abs().max())
    assert float((feat - f32).abs().max()) <= 2e-2 * fs_ + 1e-3
    # the argmax actions of a greedy policy agree wherever the reference's margin is clear
    top2 = q32.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.05 * scale
    assert bool((q.argmax(1)[clear] == q32.argmax(1)[clear]).all())


@pytest.mark.gpu
def test_dqn_rejects_non_uint8():
    from marlenv.dqn import DQNForward
    ref = RefDQN(11, 11, 8, 3).cuda()
    net = DQNForward(ref, 11, 11, 8, 3)
    with pytest.raises(TypeError):
        net(torch.zeros((2, 11, 11, 8), device='cuda'))


@pytest.mark.gpu
def test_dqn_full_batch_sampled():
    """The bench's batch (65 536 envs x 4 snakes = 262 144 observations, every
    persistent workgroup running many observations, multi-GB scratch offsets):
    512 sampled rows against the fp32 reference."""
    from marlenv.dqn import DQNForward
    torch.manual_seed(3)
    obs = _obs_batch(262144, 5, 1, seed=5)
    ref = RefDQN(11, 11, 8, 3).cuda()
    net = DQNForward(ref, 11, 11, 8, 3)
    q = net(obs)
    torch.cuda.synchronize()
    g = torch.Generator(device='cuda').manual_seed(7)
    rows = torch.cat([torch.randint(0, 262144, (508,), generator=g, device='cuda'),
                      torch.tensor([0, 1, 262142, 262143], device='cuda')])
    with torch.no_grad():
        q32 = ref(obs[rows])
    scale = float(q32.abs().max())
    assert torch.isfinite(q).all()
    assert float((q[rows] - q32).abs().max()) <= 2e-2 * scale + 1e-3


def _obs_full(B, fs=1, S=4, seed=0, H=20, W=20):
    """Full-map observations (vision_range None) of a short GPU rollout."""
    from marlenv import SnakeVecEnv
    n = max(1, -(-B // S))
    v = SnakeVecEnv(n, num_snakes=S, seed=seed, height=H, width=W, frame_stack=fs)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(seed)
    for _ in range(12):
        o, _, _, _ = v.step(torch.randint(0, 3, (n, S), generator=g, device='cuda', dtype=torch.int8))
    return o.reshape(-1, *o.shape[2:])[:B].contiguous()


@pytest.mark.gpu
@pytest.mark.parametrize('B,shape,full', [(64, (20, 20, 8), True), (37, (20, 20, 16), True), (1, (20, 20, 8), True),
                                          (300, (11, 11, 8), False), (50, (11, 11, 32), False),
                                          (20, (12, 10, 8), True), (3, (48, 48, 8), True)])
def test_dqn_fp32_matches_reference(B, shape, full):
    """precision='fp32' against the reference network in float64 on the CPU,
    |err| <= 1e-5 * max|q| (train_dqn.py's own Config: 20x20x8 full map). The
    48x48 map is wider than the matrix-core convolutions' LDS patch holds: its
    convolutions take the vector-ALU GEMM (dqn32_kernels.hip)."""
    from marlenv.dqn import DQNForward
    h, w, c = shape
    torch.manual_seed(2)
    ref = RefDQN(h, w, c, 3)
    if full:
        obs = _obs_full(B, fs=c // 8, H=h, W=w)
    else:
        obs = _obs_batch(B, (h - 1) // 2, c // 8)
    assert obs.shape == (B, h, w, c)
    net = DQNForward(ref.cuda(), h, w, c, 3, precision='fp32')
    q = net(obs)
    feat = net.forward_features(obs)
    torch.cuda.synchronize()
    ref64 = ref.double().cpu()
    with torch.no_grad():
        x = obs.cpu()
        q64 = ref64(x.double())
        f64 = ref64.forward_features(x.double())
    scale, fscale = float(q64.abs().max()), float(f64.abs().max())
    assert float((q.double().cpu() - q64).abs().max()) <= 1e-5 * scale
    assert float((feat.double().cpu() - f64).abs().max()) <= 1e-5 * fscale


@pytest.mark.gpu
def test_dqn_fp32_scales_large_inputs():
    """uint8 inputs above 1 are divided by 255 (train_dqn.py:122), as one batch."""
    from marlenv.dqn import DQNForward
    torch.manual_seed(4)
    ref = RefDQN(6, 6, 8, 2)
    g = torch.Generator(device='cuda').manual_seed(9)
    obs = torch.randint(0, 256, (9, 6, 6, 8), generator=g, device='cuda', dtype=torch.uint8)
    net = DQNForward(ref.cuda(), 6, 6, 8, 2, precision='fp32')
    q = net(obs)
    torch.cuda.synchronize()
    ref64 = ref.double().cpu()
    with torch.no_grad():
        q64 = ref64(obs.cpu().double())
    assert float((q.double().cpu() - q64).abs().max()) <= 1e-5 * float(q64.abs().max())
