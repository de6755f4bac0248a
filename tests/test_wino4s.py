"""CPU checks of the fp32 Winograd F(4x4, 3x3) transform + GEMM pipeline (csrc/kernels/wino4s_f32.hip):
the host weight transform + fragment packing (ops/conv.py wino4s_pack_np) and the kernel's V fragment order,
emulated in numpy exactly as the input transform writes V and the GEMM's MFMA steps consume both operands,
against a float64 direct convolution (the reference's Keras float32 3x3 convs, /root/reference/test/test.py:13)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C


def _emulate(x, k):
    """V as wino4s_in_kernel writes it ([tg][kc][p][lane 16 g + r][j]), M_p summed as the MFMA steps do
    (A[r][k = g] x B[k = g][n] over the 4 steps j and the chunks), y = A^T M A per tile."""
    B, H, W, Cc = x.shape
    N = k.shape[-1]
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    TG, KC = (T + 15) // 16, Cc // 16
    xp = np.zeros((B, 4 * TH + 2, 4 * TW + 2, Cc))
    xp[:, 1:H + 1, 1:W + 1] = x
    V = np.zeros((TG, KC, 36, 64, 4))
    for t in range(T):
        b, rem = divmod(t, TH * TW)
        th, tw = divmod(rem, TW)
        d = xp[b, 4 * th:4 * th + 6, 4 * tw:4 * tw + 6]
        v = np.einsum("ai,ijc,bj->abc", C.WINO4_BT, d, C.WINO4_BT).reshape(36, Cc)
        tg, r = divmod(t, 16)
        for kc in range(KC):
            for g in range(4):
                V[tg, kc, :, 16 * g + r, :] = v[:, 16 * kc + 4 * g:16 * kc + 4 * g + 4]
    U = C.wino4s_pack_np(k.astype(np.float32)).astype(np.float64)
    M = np.einsum("tkpgrj,nkpgmj->ptrnm", V.reshape(TG, KC, 36, 4, 16, 4),
                  U.reshape(N // 16, KC, 36, 4, 16, 4)).reshape(6, 6, TG * 16, N)
    Y = np.einsum("ia,abtn,jb->tijn", C.WINO4_AT, M, C.WINO4_AT)
    out = np.zeros((B, 4 * TH, 4 * TW, N))
    for t in range(T):
        b, rem = divmod(t, TH * TW)
        th, tw = divmod(rem, TW)
        out[b, 4 * th:4 * th + 4, 4 * tw:4 * tw + 4] = Y[t]
    return out[:, :H, :W]


@pytest.mark.parametrize("B,H,W,Cc,N", [(2, 7, 9, 32, 48), (1, 4, 4, 16, 16), (3, 14, 14, 16, 32),
                                        (1, 13, 6, 48, 16)])
def test_fragment_layouts_compose_to_the_convolution(B, H, W, Cc, N):
    rng = np.random.default_rng(B * H + W)
    x = rng.standard_normal((B, H, W, Cc))
    k = rng.standard_normal((3, 3, Cc, N))
    ref = F.conv2d(torch.from_numpy(x).permute(0, 3, 1, 2), torch.from_numpy(k).permute(3, 2, 0, 1),
                   padding=1).permute(0, 2, 3, 1).numpy()
    got = _emulate(x, k)
    assert np.abs(got - ref).max() / np.abs(ref).max() < 5e-6          # fp32 rounding of U only


def test_transform_matrices_are_f43():
    """B^T G / A^T of F(4x4, 3x3): A^T [(G g) * (B^T d)] == correlation of d with g for every g, d."""
    rng = np.random.default_rng(0)
    for _ in range(5):
        d, g = rng.standard_normal(6), rng.standard_normal(3)
        y = C.WINO4_AT @ ((C.WINO4_G @ g) * (C.WINO4_BT @ d))
        want = np.array([d[i:i + 3] @ g for i in range(4)])
        assert np.allclose(y, want)


def test_pack_rejects_other_filters():
    with pytest.raises(ValueError):
        C.wino4s_pack_np(np.zeros((1, 1, 16, 16), np.float32))
    with pytest.raises(ValueError):
        C.wino4s_pack_np(np.zeros((3, 3, 8, 16), np.float32))
    assert C.wino4s_splits(64) == [1, 2, 4] and C.wino4s_splits(512) == [1, 2, 4, 8] and C.wino4s_splits(16) == [1]
