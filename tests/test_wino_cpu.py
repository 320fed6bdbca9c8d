"""CPU checks of the Winograd F(4x4,3x3) algebra the fp32 kernels implement (csrc/kernels/wino.hip,
the matrices in its header and the coefficient table kWinoAT2 in conv_v2.hip): the forward
transform, the data gradient through the rot180-transposed weights, and the weight gradient by
transposition, each against a direct float64 correlation. The GPU kernels themselves are tested
against torch float64 in tests/test_wino_gpu.py."""
import numpy as np

BT = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
               [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], dtype=np.float64)
G = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
              [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], dtype=np.float64)
AT = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]],
              dtype=np.float64)


def _corr_tile(d, g):
    """4x4 output of the 3x3 correlation of a 6x6 input tile."""
    return np.array([[(d[i:i + 3, j:j + 3] * g).sum() for j in range(4)] for i in range(4)])


def test_forward_tile_identity():
    rng = np.random.default_rng(0)
    for _ in range(5):
        d, g = rng.standard_normal((6, 6)), rng.standard_normal((3, 3))
        y = AT @ ((G @ g @ G.T) * (BT @ d @ BT.T)) @ AT.T
        assert np.abs(y - _corr_tile(d, g)).max() < 1e-12


def _conv3x3(x, w):
    """x [C][H][W], w [K][C][3][3], pad 1 -> [K][H][W] (float64 reference)."""
    c, h, wd = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)))
    out = np.zeros((w.shape[0], h, wd))
    for i in range(h):
        for j in range(wd):
            out[:, i, j] = np.einsum("kcrs,crs->k", w, xp[:, i:i + 3, j:j + 3])
    return out


def _wino_conv(x, w):
    """The kernels' forward: tiles of 4x4 outputs from 6x6 windows at (4ti-1, 4tj-1)."""
    c, h, wd = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)))
    U = np.einsum("ar,kcrs,bs->kcab", G, w, G)
    out = np.zeros((w.shape[0], h, wd))
    for ti in range(h // 4):
        for tj in range(wd // 4):
            V = np.einsum("ar,crs,bs->cab", BT, xp[:, 4 * ti:4 * ti + 6, 4 * tj:4 * tj + 6], BT)
            M = np.einsum("cab,kcab->kab", V, U)
            out[:, 4 * ti:4 * ti + 4, 4 * tj:4 * tj + 4] = np.einsum("ia,kab,jb->kij", AT, M, AT)
    return out


def test_forward_and_data_gradient():
    rng = np.random.default_rng(1)
    c, k, h = 3, 5, 8
    x, w = rng.standard_normal((c, h, h)), rng.standard_normal((k, c, 3, 3))
    assert np.abs(_wino_conv(x, w) - _conv3x3(x, w)).max() < 1e-10
    # data gradient: the same algorithm on dy with U' = transform of rot180(w)^T (wino_w flip)
    dy = rng.standard_normal((k, h, h))
    wflip = w[:, :, ::-1, ::-1].transpose(1, 0, 2, 3)
    dx_ref = np.zeros((c, h, h))
    dyp = np.pad(dy, ((0, 0), (1, 1), (1, 1)))
    for i in range(h):
        for j in range(h):
            dx_ref[:, i, j] = np.einsum("ckrs,krs->c", wflip, dyp[:, i:i + 3, j:j + 3])
    assert np.abs(_wino_conv(dy, wflip) - dx_ref).max() < 1e-10


def test_weight_gradient_by_transposition():
    """dg = G^T [sum_t (A dy_t A^T) . (B^T d_t B)] G (A = AT^T): wino_dy_kernel + the TN GEMM +
    wino_wout_kernel."""
    rng = np.random.default_rng(2)
    c, k, h = 2, 3, 8
    x, dy = rng.standard_normal((c, h, h)), rng.standard_normal((k, h, h))
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)))
    ref = np.zeros((k, c, 3, 3))
    for r in range(3):
        for s in range(3):
            ref[:, :, r, s] = np.einsum("khw,chw->kc", dy, xp[:, r:r + h, s:s + h])
    M = np.zeros((k, c, 6, 6))
    for ti in range(h // 4):
        for tj in range(h // 4):
            V = np.einsum("ar,crs,bs->cab", BT, xp[:, 4 * ti:4 * ti + 6, 4 * tj:4 * tj + 6], BT)
            D = np.einsum("ai,kij,bj->kab", AT.T, dy[:, 4 * ti:4 * ti + 4, 4 * tj:4 * tj + 4], AT.T)
            M += np.einsum("kab,cab->kcab", D, V)
    dw = np.einsum("ar,kcab,bs->kcrs", G, M, G)
    assert np.abs(dw - ref).max() < 1e-10


def test_output_coefficient_table():
    """conv_v2.hip kWinoAT2[b][4 i + j] = A^T[i][r] A^T[j][s], b = 6 r + s: folding the 36 batch
    products with it equals A^T P A."""
    coef = np.array([[AT[i, b // 6] * AT[j, b % 6] for i in range(4) for j in range(4)] for b in range(36)])
    P = np.random.default_rng(3).standard_normal((6, 6))
    y = (coef * P.reshape(36, 1)).sum(0).reshape(4, 4)
    assert np.abs(y - AT @ P @ AT.T).max() < 1e-12
