"""GPU tests of the Cayley inverse (fiode_batched_inverse + block Gauss-Jordan) against
torch.linalg.inv in float64 on the same positive-real systems I + A, A = U - U^H + V^H V.

Tolerance: max |inv - inv64| <= 2e-5 * n^0.5 (||inv||_2 <= 1 for these systems, so absolute
error is the meaningful scale; fp32 Gauss-Jordan error grows ~ sqrt(n) eps ||M||)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _system(batch, n, dtype, dev, scale=1.0, tall=16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    W = torch.randn(batch, n + tall, n, generator=g, dtype=torch.float64 if dtype == torch.float32 else torch.complex128)
    W = W * scale / (n ** 0.5)
    U, V = W[:, :n], W[:, n:]
    M = torch.eye(n, dtype=W.dtype) + U - U.mH + V.mH @ V
    return M.to(dev)


@pytest.mark.parametrize("n", [1, 3, 10, 16, 17, 32, 64, 100, 128])
@pytest.mark.parametrize("dtype", [torch.float32, torch.complex64])
def test_batched_inverse_matches_float64(n, dtype):
    from fiode_amd import ops
    dev = _dev()
    M64 = _system(7, n, dtype, dev, scale=3.0, seed=n)
    ref = torch.linalg.inv(M64)
    inv = ops.batched_inverse(M64.to(dtype))
    err = float((inv.to(ref.dtype) - ref).abs().max())
    assert err <= 2e-5 * n ** 0.5, err


@pytest.mark.parametrize("n", [200, 512])
def test_block_inverse_large(n):
    from fiode_amd.cayley import _block_inverse
    dev = _dev()
    M64 = _system(2, n, torch.float32, dev, scale=2.0, seed=n)
    ref = torch.linalg.inv(M64)
    inv = _block_inverse(M64.float())
    err = float((inv.double() - ref).abs().max())
    assert err <= 2e-5 * n ** 0.5, err


@pytest.mark.parametrize("n", [65, 128, 130, 512])
def test_panel_block_inverse_kernel(n):
    """fiode_block_inverse (64-wide panels, padded with I) vs float64 torch.linalg.inv; in == out."""
    from fiode_amd import ops
    dev = _dev()
    M64 = _system(1, n, torch.float32, dev, scale=3.0, seed=n)[0]
    ref = torch.linalg.inv(M64)
    inv = ops.block_inverse(M64.float())
    assert float((inv.double() - ref).abs().max()) <= 2e-5 * n ** 0.5
    buf = M64.float().clone()
    ops.block_inverse(buf, out=buf)
    assert torch.equal(buf, inv)


def test_inverse_in_place_and_strided_batch():
    from fiode_amd import ops
    dev = _dev()
    M = _system(5, 24, torch.float32, dev, seed=3).float()
    ref = torch.linalg.inv(M.double())
    out = M.clone()
    ops.batched_inverse(out, out=out)
    assert float((out.double() - ref).abs().max()) < 2e-4


@pytest.mark.parametrize("shape", [(32, 3), (512, 4096), (512, 512), (10, 512), (128, 10), (128, 128)])
def test_cayley_orthogonal(shape):
    from fiode_amd.cayley import cayley
    dev = _dev()
    W = torch.randn(*shape, device=dev)
    Q = cayley(W / W.norm() * 3.0)
    if shape[0] >= shape[1]:
        G = Q.T @ Q
    else:
        G = Q @ Q.T
    err = float((G - torch.eye(G.shape[0], device=dev)).abs().max())
    assert err < 5e-5, err


def test_cayley_complex_batch_orthogonal():
    from fiode_amd.cayley import cayley
    dev = _dev()
    W = torch.randn(144, 32, 128, dtype=torch.complex64, device=dev)
    Q = cayley(W * 0.2)                 # wide: through the transpose
    G = Q @ Q.mH
    err = float((G - torch.eye(32, device=dev)).abs().max())
    assert err < 5e-5, err


@pytest.mark.parametrize("dtype,n", [(torch.float32, 20), (torch.float32, 300), (torch.complex64, 24)])
def test_cayley_inverse_gradient_matches_linalg_inv(dtype, n):
    from fiode_amd.cayley import _CayleyInverse
    dev = _dev()
    M = _system(3, n, dtype, dev, scale=1.5, seed=11).to(dtype)
    G = torch.randn(M.shape, dtype=dtype, device=dev)
    a = M.clone().requires_grad_(True)
    (_CayleyInverse.apply(a) * G.conj()).real.sum().backward() if dtype.is_complex else \
        (_CayleyInverse.apply(a) * G).sum().backward()
    b = M.clone().double() if not dtype.is_complex else M.clone().to(torch.complex128)
    b.requires_grad_(True)
    Gb = G.to(b.dtype)
    (torch.linalg.inv(b) * Gb.conj()).real.sum().backward() if dtype.is_complex else \
        (torch.linalg.inv(b) * Gb).sum().backward()
    err = float((a.grad.to(b.dtype) - b.grad).abs().max())
    assert err < 1e-4 * n ** 0.5, err


def test_inverse_rejects_bad_inputs():
    from fiode_amd import ops
    dev = _dev()
    with pytest.raises(ValueError):
        ops.batched_inverse(torch.eye(129, device=dev))
    with pytest.raises(TypeError):
        ops.batched_inverse(torch.eye(4, device=dev, dtype=torch.float64))
    with pytest.raises(ValueError):
        ops.batched_inverse(torch.eye(4))


@pytest.mark.parametrize("shape", [(128, 32, 32, 32), (5, 64, 8, 8), (128, 512), (3, 8)])
def test_groupsort_matches_torch_ops(shape):
    """fiode_groupsort_* vs torch.maximum/minimum + cat and their autograd (ties included)."""
    from fiode_amd.cayley import GroupSort
    dev = _dev()
    x = torch.randn(*shape, device=dev)
    x = torch.where(torch.rand_like(x) < 0.05, torch.zeros_like(x), x)      # ties between halves
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    y = GroupSort()(xa)
    a, b = xb.split(shape[1] // 2, 1)
    ref = torch.cat([torch.maximum(a, b), torch.minimum(a, b)], dim=1)
    assert torch.equal(y, ref)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    assert torch.equal(xa.grad, xb.grad)


def _cayley_autograd_reference(W, alpha, per_matrix):
    """The op-by-op formula through torch.linalg.inv (float64), differentiated by autograd."""
    if per_matrix:
        n = torch.linalg.vector_norm(W, dim=(-2, -1), keepdim=True)
        X = alpha.reshape(n.shape) * W / n
    else:
        X = alpha * W / W.norm()
    wide = X.shape[-1] > X.shape[-2]
    if wide:
        X = X.mT
    cin = X.shape[-1]
    U, V = X[..., :cin, :], X[..., cin:, :]
    eye = torch.eye(cin, dtype=X.dtype, device=X.device)
    inv = torch.linalg.inv(eye + U - U.mH + V.mH @ V)
    Q = torch.cat([inv @ (eye - (U - U.mH + V.mH @ V)), -2.0 * (V @ inv)], dim=-2)
    return Q.mT if wide else Q


@pytest.mark.parametrize("shape,dtype,per_matrix", [
    ((128, 10), torch.float32, False), ((10, 128), torch.float32, False), ((128, 128), torch.float32, False),
    ((512, 4096), torch.float32, False), ((3, 128, 10), torch.float32, True),
    ((144, 32, 128), torch.complex64, False), ((40, 64, 64), torch.complex64, False),
    ((544, 32, 3), torch.complex64, False)])
def test_cayley_scaled_forward_backward(shape, dtype, per_matrix):
    """_CayleyScaledFn (one node, analytic backward) vs autograd of the plain formula in float64."""
    from fiode_amd.cayley import cayley_scaled
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    W = torch.randn(shape, generator=g, dtype=torch.complex64 if dtype.is_complex else torch.float32).to(dev)
    nb = shape[0] if per_matrix else 1
    alpha = (torch.rand(nb, generator=g) * 3 + 0.5).to(dev)
    Wa, aa = W.clone().requires_grad_(True), alpha.clone().requires_grad_(True)
    Q = cayley_scaled(Wa, aa, per_matrix)
    wdt = torch.complex128 if dtype.is_complex else torch.float64
    Wb, ab = W.to(wdt).requires_grad_(True), alpha.double().requires_grad_(True)
    Qr = _cayley_autograd_reference(Wb, ab, per_matrix)
    assert float((Q.to(wdt) - Qr).abs().max()) < 2e-5
    G = torch.randn(Q.shape, generator=g, dtype=Q.dtype).to(dev)
    (Q * G.conj()).real.sum().backward() if dtype.is_complex else (Q * G).sum().backward()
    (Qr * G.to(wdt).conj()).real.sum().backward() if dtype.is_complex else (Qr * G.to(wdt)).sum().backward()
    for got, ref in ((Wa.grad, Wb.grad), (aa.grad, ab.grad)):
        scale = float(ref.abs().max()) + 1e-12
        assert float((got.to(ref.dtype) - ref).abs().max()) / scale < 1e-4


def test_spatial_major_backbone_matches_nchw():
    """KWLargeConcat on the spatial-major path (forward_hwcb, DC-folded bias, groupsort on dim 2)
    = the module-by-module NCHW path, forward and parameter gradients."""
    from fiode_amd.models import make_ortho_KWLarge_Concat
    dev = _dev()
    torch.manual_seed(0)
    bb = make_ortho_KWLarge_Concat(out_dim=10, act="GroupSort").to(dev).train()
    x = torch.rand(8, 3, 32, 32, device=dev)
    bb[1].spatial_major = False
    y0 = bb(x)                      # also initialises the conv alphas
    bb.zero_grad()
    y0 = bb(x)
    y0.square().sum().backward()
    g0 = [p.grad.clone() for p in bb.parameters()]
    bb.zero_grad()
    bb[1].spatial_major = True
    y1 = bb(x)
    y1.square().sum().backward()
    assert float((y1 - y0).abs().max()) < 1e-4 * (float(y0.abs().max()) + 1)
    for a, b in zip(bb.parameters(), g0):
        assert float((a.grad - b).abs().max()) <= 1e-3 * (float(b.abs().max()) + 1e-6)


def test_normalized_backbone_fused_input_bit_identical():
    """NormalizedBackbone: the first conv's transform reading the raw NCHW input and normalising on
    load (fiode_sconv_rfft2_nchw) = Normalize's spatial-major kernel + the transform, and the last
    conv writing NCHW (its GroupSort-backward transform reading NCHW) = the permute copies, bit for
    bit (forward and every parameter gradient)."""
    from fiode_amd.models import make_ortho_KWLarge_Concat
    dev = _dev()
    torch.manual_seed(1)
    bb = make_ortho_KWLarge_Concat(out_dim=10, act="GroupSort").to(dev).train()
    x = torch.rand(12, 3, 32, 32, device=dev)
    bb(x)                           # alpha init
    outs = []
    for fused in (False, True):
        bb.fused_input = fused
        bb[1].nchw_last = fused     # and the last conv writing the flatten's NCHW order directly
        bb.zero_grad()
        y = bb(x)
        y.square().sum().backward()
        outs.append((y.detach().clone(), [p.grad.clone() for p in bb.parameters()]))
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert torch.equal(a, b)


# ---- fused spectral Cayley map of CayleyConv (spectral.hip) ---------------------------------------
# (cout, cin, n): the four KWLarge convs (cin after the stride-2 space-to-channel) + square / tall /
# small-K cases.  Reference: CayleyConv.spectral_weight_reference (rfft2 + shift + conj +
# cayley_scaled, PyTorch ops) in float64 -- the formula the fused kernels restate.
SPECTRAL_CASES = [(32, 3, 32), (32, 128, 16), (64, 32, 16), (64, 256, 8), (16, 16, 8), (40, 8, 6)]


def _spectral_pair(cout, cin, n, dev, seed):
    from fiode_amd.cayley import CayleyConv
    torch.manual_seed(seed)
    conv = CayleyConv(cin, cout, 3).to(dev)
    with torch.no_grad():
        conv.alpha.fill_(float(conv.spectral_weight_reference(n, dev).detach().abs().pow(2).sum().sqrt()) * 1.7)
    conv._alpha_init = True
    ref = CayleyConv(cin, cout, 3).to(dev).double()
    ref.load_state_dict(conv.state_dict())
    ref._shift = {}
    return conv, ref


def _ref_shift(conv, n, dev):
    import math
    s = -((conv.weight.shape[2] - 1) // 2)
    k = torch.arange(n, device=dev, dtype=torch.float64)
    sh = torch.exp(2j * math.pi * s * (k[None, :] + k[:, None]) / n)[:, : n // 2 + 1]
    return sh.reshape(n * (n // 2 + 1), 1, 1)


def _spectral_ref64(ref, n, dev):
    """float64 spectral Q of the reference formula (shift kept in complex128)."""
    from fiode_amd.cayley import cayley_scaled
    cout, cin = ref.weight.shape[:2]
    nf = n * (n // 2 + 1)
    wf = torch.fft.rfft2(ref.weight, (n, n)).reshape(cout, cin, nf).permute(2, 0, 1).conj()
    wf = _ref_shift(ref, n, dev) * wf
    # cayley_scaled in float64 via the op-by-op formula (torch.linalg.inv)
    X = wf * (ref.alpha / torch.linalg.vector_norm(wf))
    wide = X.shape[-1] > X.shape[-2]
    if wide:
        X = X.mT
    k = X.shape[-1]
    U, V = X[..., :k, :], X[..., k:, :]
    M = torch.eye(k, dtype=X.dtype, device=dev) + U - U.mH + V.mH @ V
    inv = torch.linalg.inv(M)
    Q = torch.cat([2 * inv - torch.eye(k, dtype=X.dtype, device=dev), -2 * V @ inv], dim=-2)
    return Q.mT if wide else Q


@pytest.mark.parametrize("case", SPECTRAL_CASES)
def test_spectral_cayley_forward_matches_reference(case):
    cout, cin, n = case
    dev = _dev()
    conv, ref = _spectral_pair(cout, cin, n, dev, seed=cout + cin + n)
    Q = conv.spectral_weight(n, dev)
    assert Q.dtype == torch.complex64 and tuple(Q.shape) == (n * (n // 2 + 1), cout, cin)
    Q64 = _spectral_ref64(ref, n, dev)
    err = float((Q.to(torch.complex128) - Q64).abs().max())
    assert err <= 2e-5 * min(cout, cin) ** 0.5, err
    # the fused path and the op-by-op float32 path agree too
    Q32 = conv.spectral_weight_reference(n, dev)
    assert float((Q - Q32).abs().max()) <= 4e-5 * min(cout, cin) ** 0.5


@pytest.mark.parametrize("case", SPECTRAL_CASES)
def test_spectral_cayley_backward_matches_autograd(case):
    cout, cin, n = case
    dev = _dev()
    conv, ref = _spectral_pair(cout, cin, n, dev, seed=7 * cout + cin + n)
    nf = n * (n // 2 + 1)
    g = torch.Generator(device="cpu").manual_seed(n)
    G = torch.randn(nf, cout, cin, 2, generator=g, dtype=torch.float64)
    G = torch.view_as_complex(G).to(dev)
    Q = conv.spectral_weight(n, dev)
    (Q.to(torch.complex128) * G.conj()).real.sum().backward()
    Q64 = _spectral_ref64(ref, n, dev)
    (Q64 * G.conj()).real.sum().backward()
    for name in ("weight", "alpha"):
        a, b = getattr(conv, name).grad.double(), getattr(ref, name).grad
        tol = 2e-4 * float(b.abs().max())
        assert float((a - b).abs().max()) <= tol, (name, float((a - b).abs().max()), tol)


def test_spectral_cayley_orthogonal_and_rejects():
    from fiode_amd import ops
    dev = _dev()
    conv, _ = _spectral_pair(64, 256, 8, dev, seed=1)
    Q = conv.spectral_weight(8, dev)                       # [40, 64, 256]: orthonormal rows
    eye = torch.eye(64, dtype=torch.complex64, device=dev)
    assert float((Q @ Q.mH - eye).abs().max()) < 1e-4
    assert not ops.spectral_supported((8, 8, 5, 5), 16)     # 5x5 taps: not fused
    assert not ops.spectral_supported((128, 128, 3, 3), 16)  # K > 64
    with pytest.raises(ValueError):
        ops.spectral_cayley_forward(torch.zeros(8, 8, 5, 5, device=dev), torch.ones(1, device=dev), 16)


# ---- spectral conv transforms (sconv.hip) ------------------------------------------------------------
# (cin, cout, stride, input size): the four KWLarge convs + a non-GroupSort / odd-batch case.
SCONV_CASES = [(3, 32, 1, 32, True, 128), (32, 32, 2, 32, True, 128), (32, 64, 1, 16, True, 16),
               (64, 64, 2, 16, True, 24), (8, 6, 1, 8, False, 5), (2, 6, 1, 16, False, 5), (4, 8, 1, 8, True, 9)]


@pytest.mark.parametrize("case", SCONV_CASES)
def test_spectral_conv_fused_matches_torch_fft(case):
    """CayleyConv.forward_hwcb_fused (HIP rfft2 / irfft2 + GroupSort around the complex GEMMs) vs
    the torch.fft path (forward_hwcb + GroupSort) in float64, forward and every gradient."""
    from fiode_amd.cayley import CayleyConv
    cin, cout, stride, size, gs, B = case
    dev = _dev()
    torch.manual_seed(cin + cout + size)
    conv = CayleyConv(cin, cout, 3, stride=stride).to(dev)
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    n = size // stride
    conv.spectral_weight(n, dev)                        # alpha init
    ref = CayleyConv(cin, cout, 3, stride=stride).to(dev).double()
    ref.load_state_dict(conv.state_dict())
    x = torch.randn(size, size, cin, B, device=dev)
    g = torch.randn(n, n, cout, B, device=dev, dtype=torch.float64)
    xa = x.clone().requires_grad_(True)
    y = conv.forward_hwcb_fused(xa, gs)
    code = y.grad_fn.saved_tensors[2] if gs else None      # the device's GroupSort decisions
    (y.double() * g).sum().backward()
    xb = x.double().requires_grad_(True)
    xr = xb
    if stride == 2:
        h, w, c, bb = xr.shape
        xr = xr.reshape(h // 2, 2, w // 2, 2, c, bb).permute(0, 2, 4, 1, 3, 5).reshape(h // 2, w // 2, c * 4, bb)
    nf = n * (n // 2 + 1)
    xf = torch.fft.rfft2(xr, dim=(0, 1)).reshape(nf, xr.shape[2], B)
    yf = _spectral_ref64(ref, n, dev) @ xf
    yf = torch.cat([yf[:1] + (float(n * n) * ref.bias)[:, None], yf[1:]])
    yr = torch.fft.irfft2(yf.reshape(n, n // 2 + 1, cout, B), s=(n, n), dim=(0, 1))
    if gs:
        # GroupSort routed by the device's codes: at a near tie (a few of the ~10^6 pairs) float32 and
        # float64 may order the pair differently, which moves that pixel's gradient to the other
        # channel; the codes themselves must agree wherever the float64 gap is clear
        a, b = yr.split(cout // 2, 2)
        sure = (a - b).abs() > 1e-4 * (float(yr.abs().max()) + 1)
        assert torch.equal(code[sure].long(), (a <= b)[sure].long())
        gt, lt = code == 0, code == 1
        mid = (a + b) / 2
        yr = torch.cat([torch.where(gt, a, torch.where(lt, b, mid)), torch.where(gt, b, torch.where(lt, a, mid))],
                       dim=2)
    (yr * g).sum().backward()
    assert float((y.double() - yr).abs().max()) <= 2e-5 * (float(yr.abs().max()) + 1)
    for name, p, q in [("x", xa, xb), ("weight", conv.weight, ref.weight), ("alpha", conv.alpha, ref.alpha),
                       ("bias", conv.bias, ref.bias)]:
        d, r = p.grad.double(), q.grad
        assert float((d - r).abs().max()) <= 2e-4 * (float(r.abs().max()) + 1e-6), name


# (F, M, N, K, conj_trans_a): the four KWLarge layers' forward products, the three input-gradient
# products, and ragged / tiny shapes (partial tiles, K not a multiple of 4, K = 0)
# (F, M, N, K, op): "n" C = A B, "ca" C = A^H B, "cb" C = w A B^H (the weight gradient, scaled)
CGEMM_CASES = [(544, 32, 128, 3, "n"), (144, 32, 128, 128, "n"), (144, 64, 128, 32, "n"),
               (40, 64, 128, 256, "n"), (144, 128, 128, 32, "ca"), (144, 32, 128, 64, "ca"),
               (40, 256, 128, 64, "ca"), (40, 64, 256, 128, "cb"), (544, 32, 3, 128, "cb"), (144, 32, 128, 128, "cb"),
               (3, 33, 7, 70, "n"), (5, 17, 40, 5, "ca"), (4, 19, 45, 37, "cb"), (1, 1, 1, 1, "n"),
               (2, 8, 4, 0, "n")]


@pytest.mark.parametrize("case", CGEMM_CASES)
def test_cgemm_matches_complex128(case):
    """fiode_cgemm (cgemm.hip, the spectral convs' per-frequency products) vs torch.matmul in
    complex128: C[f] = A[f] B[f], A[f]^H B[f] or w[f] A[f] B[f]^H."""
    from fiode_amd import ops
    F, M, N, K, op = case
    ca, cb = op == "ca", op == "cb"
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(F * 131 + M * 7 + K)
    A = torch.randn((F, K, M) if ca else (F, M, K), dtype=torch.complex64, generator=g)
    B = torch.randn((F, N, K) if cb else (F, K, N), dtype=torch.complex64, generator=g)
    w = torch.rand(F, generator=g) + 0.5 if cb else None
    C = ops.cgemm(A.to(dev), B.to(dev), conj_trans_a=ca, conj_trans_b=cb,
                  scale=None if w is None else w.to(dev)).cpu()
    ref = (A.cdouble().mH if ca else A.cdouble()) @ (B.cdouble().mH if cb else B.cdouble())
    if w is not None:
        ref = ref * w.double()[:, None, None]
    assert C.shape == (F, M, N)
    err = float((C.cdouble() - ref).abs().max()) if C.numel() else 0.0
    assert err <= 2e-6 * (K + 1) ** 0.5 * 4, err


@pytest.mark.parametrize("K,n,C,B,gs,nchw", [(3, 32, 32, 128, True, False), (3, 32, 32, 128, True, True),
                                              (1, 8, 6, 5, False, False), (2, 16, 4, 9, True, False),
                                              (4, 8, 10, 3, False, True)])
def test_sconv_irfft2_qx_matches_gemm_then_irfft2(K, n, C, B, gs, nchw):
    """fiode_sconv_irfft2_qx (Q X formed in the inverse transform's loads) = fiode_cgemm then
    fiode_sconv_irfft2, within float32 rounding; the GroupSort codes equal where the pair is not
    within rounding of a tie."""
    from fiode_amd import ops
    dev = _dev()
    nf = n * (n // 2 + 1)
    g = torch.Generator(device="cpu").manual_seed(K * 100 + n + C)
    Q = torch.randn(nf, C, K, dtype=torch.complex64, generator=g).to(dev)
    X = torch.randn(nf, K, B, dtype=torch.complex64, generator=g).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    y1, c1 = ops.sconv_irfft2_qx(Q, X, n, B, bias=bias, groupsort=gs, nchw=nchw)
    y0, c0 = ops.sconv_irfft2(ops.cgemm(Q, X), n, C, B, bias=bias, groupsort=gs, nchw=nchw)
    assert y1.shape == y0.shape
    assert float((y1 - y0).abs().max()) <= 1e-5 * (float(y0.abs().max()) + 1)
    if gs:       # codes equal wherever the pair is not a tie within rounding
        h = C // 2
        gap = (y0[:, :h] - y0[:, h:]) if nchw else (y0[:, :, :h] - y0[:, :, h:])
        sure = gap.abs() > 1e-4
        assert torch.equal(c1[sure], c0[sure])


@pytest.mark.parametrize("B,K,J,bias", [(128, 512, 10, True), (5, 64, 16, False), (7, 130, 3, True)])
def test_head_out_kernels_match_torch(B, K, J, bias):
    """fiode_head_out = addmm and fiode_head_out_backward_gs = GroupSort backward of g Q (float64
    references), including exact ties in the GroupSort input (gradient split in half)."""
    from fiode_amd import ops
    dev = _dev()
    g0 = torch.Generator(device="cpu").manual_seed(B + K + J)
    z = torch.randn(B, K, generator=g0).to(dev)
    Q = torch.randn(J, K, generator=g0).to(dev)
    b = torch.randn(J, generator=g0).to(dev) if bias else None
    out = ops.head_out(z, Q, b)
    ref = z.double() @ Q.double().t() + (b.double() if bias else 0)
    assert float((out.double() - ref).abs().max()) <= 1e-5 * (float(ref.abs().max()) + 1)
    y = torch.randn(B, K, generator=g0).to(dev)
    y[:, 0] = y[:, K // 2]                                   # exact ties
    g = torch.randn(B, J, generator=g0).to(dev)
    gx = ops.head_out_backward_gs(g, Q, y)
    d = g.double() @ Q.double()
    h = K // 2
    a, c = y[:, :h], y[:, h:]
    da, dc = d[:, :h], d[:, h:]
    ga = torch.where(a > c, da, torch.where(a < c, dc, da / 2 + dc / 2))
    gc = torch.where(c > a, da, torch.where(c < a, dc, da / 2 + dc / 2))
    rg = torch.cat([ga, gc], 1)
    assert float((gx.double() - rg).abs().max()) <= 1e-5 * (float(rg.abs().max()) + 1)
    assert torch.equal(ops.head_out(z, Q, b), out)                      # fixed-order reduction


def test_sconv_rejects_bad_shapes():
    from fiode_amd import ops
    from fiode_amd._lib import FiodeError
    dev = _dev()
    with pytest.raises(FiodeError, match="unsupported shape"):
        ops.sconv_rfft2(torch.zeros(64, 64, 3, 4, device=dev), 64, 3, 4)      # n > 32
    with pytest.raises(FiodeError, match="unsupported shape"):   # space-to-channel needs C % 4 == 0
        ops.sconv_irfft2(torch.zeros(8 * 5, 6, 4, dtype=torch.complex64, device=dev), 8, 6, 4, downsample=True)
    with pytest.raises(ValueError):
        ops.sconv_irfft2(torch.zeros(8 * 5, 6, 3, dtype=torch.complex64, device=dev), 8, 6, 4)   # wrong B
    with pytest.raises(FiodeError, match="unsupported shape"):   # the fused product takes K <= 4
        ops.sconv_irfft2_qx(torch.zeros(8 * 5, 6, 5, dtype=torch.complex64, device=dev),
                            torch.zeros(8 * 5, 5, 4, dtype=torch.complex64, device=dev), 8, 4)


@pytest.mark.parametrize("shape,per_matrix", [((512, 4096), False), ((4096, 512), False), ((512, 512), False),
                                              ((3, 128, 10), True)])
def test_dense_cayley_fused_matches_op_by_op(shape, per_matrix):
    """_DenseCayleyFn (dense.hip stages + library GEMMs) = _CayleyScaledFn (torch ops) in float32."""
    from fiode_amd.cayley import _CayleyScaledFn, _DenseCayleyFn
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(7)
    W = torch.randn(shape, generator=g).to(dev)
    nb = shape[0] if per_matrix else 1
    alpha = (torch.rand(nb, generator=g) * 3 + 0.5).to(dev)
    G = torch.randn(shape, generator=g).to(dev)
    out = []
    for fn in (lambda w, a: _DenseCayleyFn.apply(w, a), lambda w, a: _CayleyScaledFn.apply(w, a, per_matrix)):
        Wa, aa = W.clone().requires_grad_(True), alpha.clone().requires_grad_(True)
        Q = fn(Wa, aa)
        (Q * G).sum().backward()
        out.append((Q.detach(), Wa.grad, aa.grad))
    for a, b in zip(*out):
        assert float((a - b).abs().max()) <= 1e-4 * (float(b.abs().max()) + 1e-6)


@pytest.mark.parametrize("shape", [(10, 512), (512, 10), (3, 128, 10), (2, 10, 128), (16, 16), (10, 819), (5, 7)])
def test_small_cayley_kernel_matches_dense_path(shape):
    """_SmallCayleyFn (small_cayley.hip, one workgroup per matrix) = _CayleyScaledFn (torch ops) in
    float32, forward and backward; Q has orthonormal columns (rows for wide maps)."""
    from fiode_amd.cayley import _CayleyScaledFn, _SmallCayleyFn
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    W = torch.randn(shape, generator=g).to(dev)
    per_matrix = len(shape) == 3
    nb = shape[0] if per_matrix else 1
    alpha = (torch.rand(nb, generator=g) * 3 + 0.5).to(dev)
    G = torch.randn(shape, generator=g).to(dev)
    out = []
    for fn in (lambda w, a: _SmallCayleyFn.apply(w, a), lambda w, a: _CayleyScaledFn.apply(w, a, per_matrix)):
        Wa, aa = W.clone().requires_grad_(True), alpha.clone().requires_grad_(True)
        Q = fn(Wa, aa)
        (Q * G).sum().backward()
        out.append((Q.detach(), Wa.grad, aa.grad))
    for a, b in zip(*out):
        assert float((a - b).abs().max()) <= 1e-4 * (float(b.abs().max()) + 1e-6)
    Q = out[0][0].reshape(-1, shape[-2], shape[-1])
    Qt = Q if shape[-2] >= shape[-1] else Q.mT
    eye = torch.eye(Qt.shape[-1], device=dev)
    assert float((Qt.mT @ Qt - eye).abs().max()) < 2e-5



def test_batched_block_inverse_equals_single():
    """fiode_block_inverse_batched: each matrix's result is bit-identical to its own inverse."""
    from fiode_amd import ops
    dev = _dev()
    Ms = torch.stack([_system(1, n, torch.float32, dev, scale=3.0, seed=s)[0] for s, n in ((1, 192), (2, 192),
                                                                                          (3, 192))]).float()
    inv = ops.block_inverse(Ms)
    for i in range(3):
        assert torch.equal(inv[i], ops.block_inverse(Ms[i].contiguous()))


@pytest.mark.parametrize("B,C,H,W,with_std", [(128, 3, 32, 32, True), (5, 3, 7, 9, True), (70, 2, 8, 8, False)])
def test_normalize_hwcb_matches_torch(B, C, H, W, with_std):
    """Normalize on ROCm (fiode_normalize_hwcb): bit-identical to (x - mu) / std, returned as an
    NCHW view of spatial-major storage (so the conv stack's permute is a no-op)."""
    from fiode_amd.models import Normalize
    dev = _dev()
    g = torch.Generator().manual_seed(B)
    x = torch.rand(B, C, H, W, generator=g).to(dev)
    mu, sd = [0.485, 0.456, 0.406][:C], ([0.225, 0.2, 0.25][:C] if with_std else None)
    n = Normalize(mu, sd).to(dev)
    y = n(x)
    ref = (x - n.mu) / n.std if with_std else x - n.mu
    assert torch.equal(y, ref)
    assert y.permute(2, 3, 1, 0).is_contiguous()


def test_conditional_block_inverse_skip_flag():
    """fiode_block_inverse_cond: with the device skip flag set every launch of the elimination
    returns at once (the output buffer keeps what the caller put there); with it clear the result
    is the unconditional inverse, bit for bit."""
    from fiode_amd import ops
    dev = _dev()
    M = _system(1, 256, torch.float32, dev, scale=3.0, seed=4)[0].float().contiguous()
    exact = ops.block_inverse(M)
    out = torch.full_like(M, 7.0)
    skip = torch.ones(1, dtype=torch.int32, device=dev)
    ops.block_inverse(M, out=out, skip=skip)
    torch.cuda.synchronize()
    assert bool((out == 7.0).all())
    skip.zero_()
    ops.block_inverse(M, out=out, skip=skip)
    assert torch.equal(out, exact)


@pytest.mark.parametrize("n,batch", [(64, 1), (128, 2), (512, 1)])
def test_dense_gemm_matches_float64(n, batch):
    """fiode_dense_gemm (the dense maps' backward products, dense.hip) = float64 matmul for every
    transpose combination, within 2e-5 of the result's max (fp32 sums over K = n)."""
    import ctypes as ct
    from fiode_amd import ops, _lib as L
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + batch)
    A = torch.randn(batch, n, n, generator=g).to(dev)
    B = torch.randn(batch, n, n, generator=g).to(dev)
    for ta in (0, 1):
        for tb in (0, 1):
            C = torch.empty_like(A)
            L.check(L.lib().fiode_dense_gemm(ops._stream(dev), batch, n, ta, tb, A.data_ptr(), B.data_ptr(),
                                             C.data_ptr()), "fiode_dense_gemm")
            a, b = A.double(), B.double()
            ref = (a.mT if ta else a) @ (b.mT if tb else b)
            err = float((C.double() - ref).abs().max())
            assert err <= 2e-5 * float(ref.abs().max()), (ta, tb, err)
    assert L.lib().fiode_dense_gemm(ops._stream(dev), 1, 96, 0, 0, A.data_ptr(), B.data_ptr(), A.data_ptr()) == \
        2      # FIODE_ESHAPE (include/fiode.h)



@pytest.mark.parametrize("shape", [(512, 512), (512, 4096), (128, 128), (1024, 256), (2, 256, 256)])
def test_dense_fused_inverse_equals_staged(shape):
    """The dense map forward with the one-launch inverse building M on load (fiode_dense_cayley_
    inverse: no prep launch, Q of a square map written by the inverse) = the staged path (prep
    kernel -> M -> fiode_block_inverse -> finish), bit for bit: Q, and dL/dW, dL/dalpha."""
    from fiode_amd import cayley as CY
    dev = _dev()
    g = torch.Generator().manual_seed(sum(shape))
    W = (torch.randn(*shape, generator=g) / shape[-1] ** 0.5).to(dev)
    alpha = (W.reshape(-1, shape[-2], shape[-1]).norm(dim=(-2, -1)) * 1.5).reshape(-1 if len(shape) == 3 else 1)
    gQ = torch.randn(*shape, generator=g).to(dev)
    out = {}
    for fused in (True, False):
        CY.DENSE_FUSED_INVERSE = fused
        try:
            Wl, al = W.clone().requires_grad_(True), alpha.clone().requires_grad_(True)
            assert CY._dense_fused_ok(Wl) == fused
            Q = CY._DenseCayleyFn.apply(Wl, al)
            (Q * gQ).sum().backward()
            torch.cuda.synchronize()
            out[fused] = (Q.detach().clone(), Wl.grad.clone(), al.grad.clone())
        finally:
            CY.DENSE_FUSED_INVERSE = True
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)
    Qt = out[True][0].reshape(-1, shape[-2], shape[-1])
    Qt = Qt if shape[-2] >= shape[-1] else Qt.mT
    eye = torch.eye(Qt.shape[-1], device=dev)
    assert float((Qt.mT @ Qt - eye).abs().max()) < 5e-5


@pytest.mark.parametrize("out_kernel,out_dim", [(True, 10), (False, 10), (True, 128)])
def test_linear_head_side_stream_wgrad_matches_autograd(out_kernel, out_dim):
    """KWLargeConcat's head as one node (_LinearHeadFn: fiode_gemm products, weight / bias gradients
    on a side stream) against the module-by-module autograd chain (F.linear + GroupSort) on the same
    inputs: output, input gradient and weight gradients within float32 rounding.  out_dim = 128
    (make_ortho_KWLarge_Concat's and ExpConfig's default; more than fiode_head_out's 16 outputs)
    takes fiode_gemm for the output layer too (it used to raise ESHAPE)."""
    from fiode_amd import cayley as cy
    from fiode_amd.models import KWLargeConcat
    dev = _dev()
    torch.manual_seed(0)
    net = KWLargeConcat(out_dim=out_dim).to(dev).train()
    mods = list(net.model)[-5:]
    h0 = torch.randn(128, 4096, device=dev)
    gout = torch.randn(128, out_dim, device=dev)
    res = {}
    cy.HEAD_OUT_KERNEL = out_kernel
    try:
        for fused in (False, True):
            cy.HEAD_WGRAD_SIDE = fused
            for m in mods:
                if isinstance(m, cy.CayleyLinear):
                    m.zero_grad(set_to_none=True)
            h = h0.clone().requires_grad_(True)
            out = cy.linear_head(mods, h)
            out.backward(gout)
            torch.cuda.synchronize()
            res[fused] = (out.detach().clone(), h.grad.clone(),
                          [p.grad.clone() for m in mods if isinstance(m, cy.CayleyLinear)
                           for p in (m.weight, m.alpha, m.bias)])
    finally:
        cy.HEAD_WGRAD_SIDE = True
        cy.HEAD_OUT_KERNEL = True
    assert torch.allclose(res[False][0], res[True][0], rtol=1e-5, atol=1e-5)
    assert torch.allclose(res[False][1], res[True][1], rtol=1e-5, atol=1e-6)
    for a, b in zip(res[False][2], res[True][2]):     # the input gradients above differ in rounding
        assert float((a - b).abs().max()) <= 1e-4 * (float(b.abs().max()) + 1e-6), float((a - b).abs().max())


def test_block_inverse_timeout_poisons_instead_of_finite_wrong():
    """k_pinv's polls are bounded; with the bound lowered to one retry most polls time out.  A
    timed-out chain workgroup publishes its pivot inverse as NaN and a timed-out tile workgroup
    poisons the tiles it hands on, so every output entry is either NaN or exactly the
    healthy launch's value -- never a finite value built from stale workspace tiles."""
    import ctypes as ct
    from fiode_amd import _lib as L
    from fiode_amd.cayley import _block_inverse
    dev = _dev()
    lib = L.lib()
    fn = lib.fiode_debug_set_pinv_spin_limit
    fn.restype, fn.argtypes = ct.c_uint, [ct.c_uint]
    g = torch.Generator(device="cpu").manual_seed(31)
    n = 512
    A = torch.randn(n, n, generator=g) / n ** 0.5
    M = (torch.eye(n) + A - A.t()).to(dev)
    ref = _block_inverse(M)
    torch.cuda.synchronize()
    fn(1)
    try:
        out = _block_inverse(M)
        torch.cuda.synchronize()
    finally:
        fn(0)
    fin = torch.isfinite(out)
    assert not bool(fin.all())                      # something timed out at this bound
    assert torch.equal(out[fin], ref[fin])
    again = _block_inverse(M)                       # the default bound is back
    torch.cuda.synchronize()
    assert torch.equal(again, ref)

