"""fp32 stem K order (`ops/conv.py stem_f32_k_order`) vs the reads the kernel
makes (`csrc/kernels/stem_f32.hip`): every one of the 147 taps exactly once,
and the (filter row, tap) each lane reads at each packed K position is the tap
the packed weight there belongs to.  The kernel's per-lane address logic is
mirrored here line by line; the numerics are pinned on the GPU by
`tests/test_fp32_gpu.py` (stem vs fp32 torch conv + max-pool)."""
import numpy as np

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C


def _kernel_reads():
    """{packed K position: (filter row, tap)} as stem_pool_f32_kernel reads them."""
    reads = {}
    for fq in range(4):
        for h in range(8):                                  # bop(h): koff = (p / 5, 4 (p % 5))
            p = 4 * h + fq
            for e in range(4):
                reads[16 * h + 4 * fq + e] = (p // 5, 4 * (p % 5) + e)
        g8 = fq == 3
        j8 = 20 if g8 else 4 * (fq + 2)
        for e in range(4):                                  # half 8
            reads[128 + 4 * fq + e] = (e if g8 else 6, j8 + (0 if g8 else e))
        reads[144 + 4 * fq] = (4 + fq if fq < 3 else 4, 20)  # last MFMA, element 0
    return reads


def test_every_tap_once():
    order = C.stem_f32_k_order()
    assert order.shape == (C.STEM_F32_K,)
    taps = order[order >= 0]
    assert sorted(taps.tolist()) == list(range(147))


def test_kernel_reads_match_packed_taps():
    order = C.stem_f32_k_order()
    reads = _kernel_reads()
    for k, tap in enumerate(order):
        if tap < 0:
            continue
        assert k in reads, f"packed position {k} holds tap {tap} but no MFMA consumes it"
        s, j = reads[k]
        assert j <= 20 and s * 21 + j == tap, (k, tap, reads[k])


def test_pack_places_weights():
    rng = np.random.default_rng(0)
    kern = rng.standard_normal((7, 7, 3, 64)).astype(np.float32)
    ps = C.pack_stem_f32(kern, np.zeros(64, np.float32), ((3, 3), (3, 3)), "cpu")
    w = ps.w.numpy()
    order = C.stem_f32_k_order()
    flat = kern.transpose(3, 0, 1, 2).reshape(64, 147)
    np.testing.assert_array_equal(w[:, order >= 0], flat[:, order[order >= 0]])
    assert not w[:, order < 0].any()
    # the dot product over the packed layout equals the plain one
    patch = rng.standard_normal(147).astype(np.float32)
    packed_patch = np.where(order >= 0, patch[np.maximum(order, 0)], 0.0)
    np.testing.assert_allclose(w @ packed_patch, flat @ patch, rtol=1e-5, atol=1e-5)
