"""Stream-K fp32 batched NT GEMM (csrc/kernels/wino_gemm.hip) against torch float64: the
Winograd shapes of ResNet-18's 8x8x256 / 4x4x512 layers (both tile widths), a ragged M (zero-page
rows), split tiles (fixup through the workspace), and bit-reproducibility across launches.
Bar: max-abs error <= 1e-5 of the reference's max-abs (exact-fp32 MFMA, K <= 512)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from psx.ops import kernels as K  # noqa: E402

DEV = "cuda"


def _case(m, n, kd, nb, bn=0, seed=0):
    torch.manual_seed(seed)
    a = torch.randn(nb, m, kd, device=DEV)
    b = torch.randn(n, nb, kd, device=DEV)
    c = torch.full((nb, m, n), float("nan"), device=DEV)
    rc = K.sk_gemm_nt(a, b, c, m, n, kd, nb, (kd, m * kd), (nb * kd, kd), (n, m * n), bn=bn)
    assert rc == 0, rc
    torch.cuda.synchronize()
    ref = torch.bmm(a.double(), b.double().permute(1, 2, 0))
    return c, ref


@pytest.mark.parametrize("m,n,kd,nb,bn", [(512, 256, 256, 36, 0), (512, 256, 256, 36, 64), (128, 512, 512, 36, 0),
                                          (128, 512, 512, 36, 128), (200, 128, 64, 5, 0), (2048, 128, 128, 36, 0),
                                          (96, 64, 96, 3, 64)])
def test_sk_gemm_vs_fp64(m, n, kd, nb, bn):
    c, ref = _case(m, n, kd, nb, bn)
    err = ((c.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-5, err


@pytest.mark.parametrize("m,n,kd,bn", [(512, 256, 256, 128), (128, 512, 512, 64), (512, 256, 256, 64)])
def test_sk_gemm_bit_reproducible(m, n, kd, bn):
    """Split tiles hand their partials over through the L2 (same-XCD partners) or memory: every
    repeat is bit-identical and matches fp64 (a stale partial would break both)."""
    c1, ref = _case(m, n, kd, 36, bn, seed=4)
    assert ((c1.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    torch.manual_seed(4)
    a = torch.randn(36, m, kd, device=DEV)
    b = torch.randn(n, 36, kd, device=DEV)
    for _ in range(8):
        c = torch.full((36, m, n), float("nan"), device=DEV)
        assert K.sk_gemm_nt(a, b, c, m, n, kd, 36, (kd, m * kd), (36 * kd, kd), (n, m * n), bn=bn) == 0
        torch.cuda.synchronize()
        assert torch.equal(c, c1)


def test_sk_gemm_refuses_three_way_split():
    # 4x4x512 with 128-wide tiles: 144 tiles of 16 chunks over 144 workgroups is fine; a shape
    # whose tiles would span three workgroups is refused (-3), never run wrong
    torch.manual_seed(1)
    a = torch.randn(1, 128, 1024, device=DEV)
    b = torch.randn(512, 1, 1024, device=DEV)
    c = torch.empty(1, 128, 512, device=DEV)
    rc = K.sk_gemm_nt(a, b, c, 128, 512, 1024, 1, (1024, 128 * 1024), (1024, 1024), (512, 128 * 512), bn=64)
    assert rc in (0, -3)
    if rc == 0:
        torch.cuda.synchronize()
        ref = a[0].double() @ b[:, 0].double().T
        assert ((c[0].double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
