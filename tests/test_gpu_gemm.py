"""fiode_gemm (gemm.hip): the hand-written f32 GEMM that replaces torch.matmul / addmm on the Cayley
layers' products (cayley.py _dense_*, _LinearHeadFn; classification.py:282-293, models.py:29-35).

Checked against float64 torch matmul of the same float32 operands: every shape the training step
runs (the 4096 -> 512 map's V'^T V' / V' inv / backward products, the head's x Q^T + b, g Q and
g^T x), ragged shapes (M = 10 head gradient, K = 3, N = 1, tiles cut by every edge), transposed
views read in place, batches (also a 2-D operand shared by the batch), alpha / beta / bias, forced
split-K counts -- within 8 sqrt(K) ulp of the |A| |B| product -- plus bit-reproducibility of the
split-K reduction and the counter words left zero."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _check(C, A, B, alpha=1.0, beta=0.0, C0=None, bias=None):
    A64, B64 = A.double(), B.double()
    ref = alpha * (A64 @ B64)
    mag = abs(alpha) * (A64.abs() @ B64.abs())
    if C0 is not None:
        ref = ref + beta * C0.double()
        mag = mag + abs(beta) * C0.double().abs()
    if bias is not None:
        ref = ref + bias.double()
        mag = mag + bias.double().abs()
    K = A.shape[-1]
    tol = 8 * math.sqrt(max(K, 1)) * 2.0 ** -24 * mag + 1e-30
    err = (C.double() - ref).abs()
    assert bool((err <= tol).all()), float((err / (mag + 1e-30)).max())


# (M, K, N) of the configs[1] step: the 4096 -> 512 dense map's products (k = 512, R - k = 3584) and
# the KWLarge head at B = 128 (forward x Q^T, input gradient g Q, weight gradient g^T x)
STEP_SHAPES = [
    (512, 3584, 512, "A_rowmajor_B_view"),      # G = W2 W2^T   (W2 = W[:, 512:], row stride 4096)
    (512, 512, 3584, "At_B"),                   # P = inv^T W2
    (128, 4096, 512, "A_Bt"),                   # y1 = h Q1^T + b1
    (128, 512, 512, "A_Bt"),                    # y2 = z1 Q2^T + b2
    (128, 512, 4096, "A_B"),                    # dh = g1 Q1
    (512, 128, 4096, "At_B"),                   # dW1 = g1^T h
    (10, 128, 512, "At_B"),                     # dW3 = g^T z2
]


@pytest.mark.parametrize("M,K,N,form", STEP_SHAPES)
def test_step_shapes_match_float64(M, K, N, form):
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + K + N)
    if form == "A_rowmajor_B_view":
        W = torch.randn(M, K + 512, generator=g).to(dev)
        A = W[:, 512:]
        B = A.mT
    elif form == "At_B":
        A = torch.randn(K, M, generator=g).to(dev).t()
        B = torch.randn(K, N, generator=g).to(dev)
    elif form == "A_Bt":
        A = torch.randn(M, K, generator=g).to(dev)
        B = torch.randn(N, K, generator=g).to(dev).t()
    else:
        A = torch.randn(M, K, generator=g).to(dev)
        B = torch.randn(K, N, generator=g).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    C = ops.mm(A, B, bias=bias)
    torch.cuda.synchronize()
    _check(C, A, B, bias=bias)


@pytest.mark.parametrize("M,K,N", [(10, 128, 512), (1, 3, 1), (65, 33, 63), (130, 100, 70), (7, 0, 5), (64, 4, 64),
                                   (3, 257, 129), (200, 1000, 1)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_ragged_shapes_and_layouts(M, K, N, ta, tb):
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(M + 3 * K + 5 * N + ta + 2 * tb)
    A = torch.randn(K, M, generator=g).to(dev).t() if ta else torch.randn(M, K, generator=g).to(dev)
    B = torch.randn(N, K, generator=g).to(dev).t() if tb else torch.randn(K, N, generator=g).to(dev)
    C = ops.mm(A, B)
    torch.cuda.synchronize()
    _check(C, A, B)


@pytest.mark.parametrize("split", [1, 2, 3, 7, 32])
def test_forced_splits_alpha_beta(split):
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(split)
    A = torch.randn(96, 1000, generator=g).to(dev)
    B = torch.randn(1000, 80, generator=g).to(dev)
    C0 = torch.randn(96, 80, generator=g).to(dev)
    C = C0.clone()
    ops.mm(A, B, alpha=-0.5, beta=2.0, out=C, split_k=split)
    torch.cuda.synchronize()
    _check(C, A, B, alpha=-0.5, beta=2.0, C0=C0)


def test_batched_and_shared_operand():
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn(3, 70, 200, generator=g).to(dev)
    B = torch.randn(200, 90, generator=g).to(dev)
    C = ops.mm(A, B)
    Bb = torch.randn(3, 90, 200, generator=g).to(dev).mT
    C2 = ops.mm(A, Bb)
    torch.cuda.synchronize()
    for b in range(3):
        _check(C[b], A[b], B)
        _check(C2[b], A[b], Bb[b])


def test_split_k_is_bit_reproducible_and_leaves_counters_zero():
    """The partial tiles are added in split order by whichever workgroup finishes a tile last:
    repeated calls give the same bits, and every call leaves the counter words at zero."""
    from fiode_amd import ops, _lib as L
    import ctypes as ct
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(9)
    W = torch.randn(512, 4096, generator=g).to(dev)
    A = W[:, 512:]
    d = L.GemmDesc(1, 512, 512, 3584, 0, 1, 4096, 4096, 512, 0, 0, 0, 1.0, 0.0, 0)
    assert L.lib().fiode_gemm_splits(ct.byref(d)) > 1
    outs = [ops.mm(A, A.mT) for _ in range(4)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    nb = L.lib().fiode_gemm_counter_bytes(ct.byref(d))
    ws = ops._gemm_ws(dev, 0)
    assert nb > 0 and int(ws[:nb].count_nonzero()) == 0


def test_calls_of_different_shapes_share_the_workspace():
    """Every split-K call on a stream uses one workspace whose counter block sits at a fixed place:
    a call with many tiles after one with few (whose partials lay where a shape-dependent counter
    block would have grown to) still sums its tiles correctly (the first round-6 layout did not)."""
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(13)
    A1 = torch.randn(128, 4096, generator=g).to(dev)
    B1 = torch.randn(4096, 512, generator=g).to(dev)
    A2 = torch.randn(128, 512, generator=g).to(dev)
    B2 = torch.randn(512, 4096, generator=g).to(dev)
    for _ in range(2):
        C1 = ops.mm(A1, B1, split_k=16)             # 16 tiles x 16 splits
        C2 = ops.mm(A2, B2, split_k=2)              # 128 tiles x 2 splits
        C3 = ops.mm(A1, B1, split_k=3)
        torch.cuda.synchronize()
        _check(C1, A1, B1)
        _check(C2, A2, B2)
        _check(C3, A1, B1)


@pytest.mark.parametrize("M,K,N,cap", [(512, 3584, 512, 64), (512, 512, 3584, 64), (512, 512, 3584, 8),
                                       (130, 70, 90, 8), (128, 4096, 512, 16)])
def test_capped_grid_equals_full_grid(M, K, N, cap):
    """max_workgroups (a persistent grid looping over the tiles, split-K included) computes the same
    bits as one workgroup per tile: the same tiles, the same k order, the same split order."""
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(M + K + N)
    A = torch.randn(M, K, generator=g).to(dev)
    B = torch.randn(K, N, generator=g).to(dev)
    full = ops.mm(A, B)
    capped = ops.mm(A, B, max_workgroups=cap)
    torch.cuda.synchronize()
    assert torch.equal(full, capped)
    _check(capped, A, B)


@pytest.mark.parametrize("wide", [True, False])
def test_pair_equals_two_calls(wide):
    """fiode_gemm_pair (two products in one launch: the dense maps' backward A = V'^T Gb beside
    P2 = Gb inv^T) gives the same bits as the two fiode_gemm calls, for the wide map's operand views
    and the tall mirror, and shapes the one-launch kernel does not take fall back to two launches."""
    from fiode_amd import ops
    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(17 + wide)
    k, R = 512, 4096
    W = torch.randn(1, k, R, generator=g).to(dev) if wide else torch.randn(1, R, k, generator=g).to(dev)
    gQ = torch.randn_like(W)
    inv = torch.randn(1, k, k, generator=g).to(dev)
    if wide:
        Vp, Gb = W[:, :, k:].mT, gQ[:, :, k:].mT
        ops_ = (Vp.mT, Gb, inv, gQ[:, :, k:])
    else:
        Vp, Gb = W[:, k:, :], gQ[:, k:, :]
        ops_ = (Vp.mT, Gb, Gb, inv.mT)
    A0, P0 = ops.mm(ops_[0], ops_[1]), ops.mm(ops_[2], ops_[3])
    A1, P1 = ops.mm_pair(*ops_)
    torch.cuda.synchronize()
    assert torch.equal(A0, A1) and torch.equal(P0, P1)
    _check(A1[0], ops_[0][0], ops_[1][0])
    # a ragged pair (register K loop): two launches, same bits
    X, Y = torch.randn(70, 33, generator=g).to(dev), torch.randn(33, 50, generator=g).to(dev)
    r0, r1 = ops.mm_pair(X, Y, Y.t(), X.t())
    torch.cuda.synchronize()
    assert torch.equal(r0, ops.mm(X, Y)) and torch.equal(r1, ops.mm(Y.t(), X.t()))
