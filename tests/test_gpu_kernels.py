"""GPU parity of the individual HIP kernels (through the C ABI) against the oracle and
the reference's golden vectors.  Tolerances: fp32 path, relative 1e-4 on the loss
(north_star), element-wise tolerances stated per test."""
import numpy as np
import pytest
import torch

import recipe
from conftest import golden
from oracle import ge2e_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(100, 72, 40), (256, 768, 640), (3072, 40, 2048), (640, 3072, 768), (8, 4, 4),
                                   (512, 256, 8192), (512, 384, 1024)])   # 256-tile: split-K, BN = 128
def test_gemm_f32_layouts(ak, bk, M, N, K):
    from pytorch_speaker_verification_amd.ops import gemm_f32
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + ak * 2 + bk)
    A = torch.randn((M, K) if ak else (K, M), generator=g)
    B = torch.randn((N, K) if bk else (K, N), generator=g)
    ref = (A.double() if ak else A.double().T) @ (B.double().T if bk else B.double())
    C = gemm_f32(A.to(DEV), B.to(DEV), bool(ak), bool(bk)).cpu().double()
    err = (C - ref).abs().max().item()
    assert err <= 2e-6 * K ** 0.5 * ref.abs().max().item() + 1e-5, err


def _ge2e_gpu(E, w, b):
    from pytorch_speaker_verification_amd import ops
    Et = torch.tensor(E, device=DEV)
    wt = torch.tensor(w, dtype=torch.float32, device=DEV)
    bt = torch.tensor(b, dtype=torch.float32, device=DEV)
    loss, per, st = ops.ge2e_forward(Et, wt, bt)
    dE, dw, db = ops.ge2e_backward(st, wt, bt)
    return float(loss), per.cpu().numpy(), dE.cpu().numpy(), float(dw), float(db)


def test_ge2e_kat0():
    k = golden("kat0.npz")
    loss, per, dE, dw, db = _ge2e_gpu(k["E"], 1.0, 0.0)
    assert abs(loss - float(k["loss"])) <= 1e-4 * abs(float(k["loss"]))
    np.testing.assert_allclose(per, k["per"], atol=1e-5)
    np.testing.assert_allclose(dE, k["dE"], atol=1e-5)
    assert abs(dw - float(k["dw"])) < 1e-5 and abs(db - float(k["db"])) < 1e-5


@pytest.mark.parametrize("tag", ["n4m5", "n4m5_flat", "n8m10_wb", "n64m10", "n256m10", "n3m2"])
def test_ge2e_golden(tag):
    g = golden(f"ge2e_{tag}.npz")
    E = recipe.make_embeddings(int(g["seed"]), int(g["n"]), int(g["m"]), int(g["d"]), bool(g["clustered"]))
    w, b = float(g["w"]), float(g["b"])
    loss, per, dE, dw, db = _ge2e_gpu(E, w, b)
    ref_loss = float(g["loss"])
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)       # fp32 loss within 1e-4 (rel)
    np.testing.assert_allclose(per, g["per"], atol=1e-4)
    o_dE, o_dw, o_db = ge2e_np.ge2e_backward(E, w, b)
    scale = np.abs(o_dE).max()
    np.testing.assert_allclose(dE, o_dE, atol=1e-4 * scale)
    assert abs(dw - o_dw) <= 1e-4 * max(1.0, abs(o_dw))
    assert abs(db - o_db) <= 1e-5 * E.shape[0] * E.shape[1]


@pytest.mark.parametrize("tag", ["kat0", "n4m5", "n4m5_flat", "n8m10_wb", "n64m10", "n3m2", "n256m10"])
def test_ge2e_fused_train_golden(tag):
    """The fused 3-launch training form (sv_ge2e_train) against the reference's golden vectors
    and the split path: loss, per-row loss, dE, dw, db."""
    from pytorch_speaker_verification_amd import ops
    if tag == "kat0":
        k = golden("kat0.npz")
        E, w, b = k["E"], 1.0, 0.0
        ref = dict(loss=float(k["loss"]), per=k["per"], dE=k["dE"], dw=float(k["dw"]), db=float(k["db"]))
    else:
        g = golden(f"ge2e_{tag}.npz")
        E = recipe.make_embeddings(int(g["seed"]), int(g["n"]), int(g["m"]), int(g["d"]), bool(g["clustered"]))
        w, b = float(g["w"]), float(g["b"])
        o_dE, o_dw, o_db = ge2e_np.ge2e_backward(E, w, b)
        ref = dict(loss=float(g["loss"]), per=g["per"], dE=o_dE, dw=o_dw, db=o_db)
    Et = torch.tensor(E, device=DEV)
    wt = torch.tensor(w, dtype=torch.float32, device=DEV)
    bt = torch.tensor(b, dtype=torch.float32, device=DEV)
    loss, per, dE, dwdb = ops.ge2e_train(Et, wt, bt)
    loss, per, dE, dwdb = float(loss), per.cpu().numpy(), dE.cpu().numpy(), dwdb.cpu().numpy()
    sl, sper, sdE, sdw, sdb = _ge2e_gpu(E, w, b)
    assert abs(loss - ref["loss"]) <= 1e-4 * abs(ref["loss"]), (loss, ref["loss"])
    np.testing.assert_allclose(per, ref["per"], atol=1e-4)
    scale = max(np.abs(ref["dE"]).max(), 1e-30)
    np.testing.assert_allclose(dE, ref["dE"], atol=1e-4 * scale)
    assert abs(dwdb[0] - ref["dw"]) <= 1e-4 * max(1.0, abs(ref["dw"]))
    assert abs(dwdb[1] - ref["db"]) <= 1e-5 * E.shape[0] * E.shape[1]
    # against the split (MFMA-GEMM) path on the same inputs: fp32-rounding level
    d_loss = abs(loss - sl) / abs(sl)
    d_dE = float(np.abs(dE - sdE).max()) / scale
    print(f"\nMEASURED ge2e_fused_vs_split.{tag} loss_rel {d_loss:.2e} dE_rel {d_dE:.2e} fused {loss!r} split {sl!r} "
          f"golden {ref['loss']!r} per_dev {float(np.abs(per - sper).max()):.2e}")
    # per-row losses to fp32 rounding; the (sum) loss of nearly-separated speakers is tiny and
    # cancels, so it is held in absolute terms (measured: 7.6e-6 at 640 rows, dE 3.6e-6 rel)
    n_rows = E.shape[0] * E.shape[1]
    assert float(np.abs(per - sper).max()) <= 5e-6
    assert abs(loss - sl) <= 3e-6 * n_rows ** 0.5 and d_dE <= 4e-5, (d_loss, d_dE)


def test_ge2e_diagonal_index_set_exact():
    """The leave-one-out (diagonal) entries are exactly the k == j entries: perturbing
    one speaker's utterance changes only that speaker's diagonal centroid term."""
    from pytorch_speaker_verification_amd.utils import get_centroids, get_cossim
    E = recipe.make_embeddings(3, 6, 4, 256, True)
    Et = torch.tensor(E, device=DEV)
    C = get_centroids(Et)
    cos = get_cossim(Et, C).cpu().numpy()
    ref = ge2e_np.get_cossim(E, ge2e_np.get_centroids(E))
    np.testing.assert_allclose(cos, ref, atol=2e-6)
    # the diagonal differs from the plain centroid cosine everywhere (leave-one-out), off-diag equal
    plain = np.einsum("jid,kd->jik", E / np.linalg.norm(E, axis=-1, keepdims=True),
                      ge2e_np._unit(ge2e_np.get_centroids(E))[0]) + 1e-6
    diff = np.abs(cos - plain) > 1e-4
    assert np.array_equal(diff, np.broadcast_to(np.eye(6, dtype=bool)[:, None, :], diff.shape))


def test_get_cossim_external_centroids_and_calc_loss():
    from pytorch_speaker_verification_amd.utils import calc_loss, get_centroids, get_cossim
    g = golden("cossim_ext.npz")
    C = get_centroids(torch.tensor(g["enroll"], device=DEV))
    np.testing.assert_allclose(C.cpu().numpy(), g["enroll_centroids"], atol=1e-6)
    cos = get_cossim(torch.tensor(g["verif"], device=DEV), C)
    np.testing.assert_allclose(cos.cpu().numpy(), g["cossim"], atol=2e-6)
    k = golden("kat0.npz")
    S = torch.tensor(k["cossim"], device=DEV)
    loss, per = calc_loss(S)
    assert abs(float(loss) - float(k["loss"])) < 1e-4 * float(k["loss"])
    np.testing.assert_allclose(per.cpu().numpy(), k["per"], atol=1e-5)


def test_clip_sgd_matches_torch():
    from pytorch_speaker_verification_amd.ops import clip_sgd_step_
    g = torch.Generator().manual_seed(5)
    for n, max_norm in [(12134656, 3.0), (1003, 1.0), (2, 1.0), (4096, 1e6)]:
        p = torch.randn(n, generator=g)
        gr = torch.randn(n, generator=g) * 0.1
        pr, grr = p.clone().double(), gr.clone().double()
        norm = grr.norm()
        coef = min(1.0, max_norm / (float(norm) + 1e-6))
        pr -= 0.01 * coef * grr
        pd, gd = p.to(DEV), gr.to(DEV)
        out = torch.zeros(1, device=DEV)
        clip_sgd_step_(pd, gd, max_norm, 0.01, write_grad=True, norm_out=out)
        np.testing.assert_allclose(pd.cpu().double().numpy(), pr.numpy(), atol=1e-6)
        np.testing.assert_allclose(gd.cpu().double().numpy(), (grr * coef).numpy(), atol=1e-6)
        assert abs(float(out) - float(norm)) <= 1e-5 * float(norm)


@pytest.mark.parametrize("write_grad", [False, True])
@pytest.mark.parametrize("n0,n1", [(12134656, 4), (1003, 2), (4096, 8192)])
def test_clip_sgd_step2_is_two_steps(n0, n1, write_grad):
    """sv_clip_sgd_step2 (both groups in one launch pair, what the trainer runs) = two
    sv_clip_sgd_step calls, bit for bit: parameters, gradients and both norms; and the status word
    skips both groups."""
    from pytorch_speaker_verification_amd._lib import PersistStatus
    from pytorch_speaker_verification_amd.ops import clip_sgd_step2_, clip_sgd_step_
    g = torch.Generator().manual_seed(n0 + n1)
    p0, g0 = torch.randn(n0, generator=g).to(DEV), (torch.randn(n0, generator=g) * 0.1).to(DEV)
    p1, g1 = torch.randn(n1, generator=g).to(DEV), (torch.randn(n1, generator=g) * 3.0).to(DEV)
    a = [t.clone() for t in (p0, g0, p1, g1)]
    na, nb = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
    clip_sgd_step_(a[0], a[1], 3.0, 0.01, write_grad=write_grad, norm_out=na[0:1])
    clip_sgd_step_(a[2], a[3], 1.0, 0.01, write_grad=write_grad, norm_out=na[1:2])
    b = [t.clone() for t in (p0, g0, p1, g1)]
    clip_sgd_step2_(b[0], b[1], 3.0, b[2], b[3], 1.0, 0.01, write_grad=write_grad, norm_out=nb)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(na, nb)
    st = PersistStatus(torch.device(DEV))
    st.block[0] = 1  # a timed-out recurrence: nothing may change
    c = [t.clone() for t in (p0, g0, p1, g1)]
    clip_sgd_step2_(c[0], c[1], 3.0, c[2], c[3], 1.0, 0.01, write_grad=True, norm_out=nb, status=st)
    torch.cuda.synchronize()
    for x, y in zip(c, (p0, g0, p1, g1)):
        assert torch.equal(x, y)
    assert bool(torch.isnan(nb).all())


@pytest.mark.parametrize("M,N,K", [(640, 256, 768), (100, 36, 1024), (3000, 3072, 40)])
def test_gemm_f32_bias_and_split_k(M, N, K):
    """Bias epilogue on both the direct and the split-K (slab reduce) paths."""
    from pytorch_speaker_verification_amd.ops import gemm_f32
    g = torch.Generator().manual_seed(M + N + K)
    A, B, bias = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
    ref = A.double() @ B.double().T + bias.double()
    C = gemm_f32(A.to(DEV), B.to(DEV), True, True, bias=bias.to(DEV)).cpu().double()
    assert (C - ref).abs().max().item() <= 2e-6 * K ** 0.5 * ref.abs().max().item() + 1e-5


@pytest.mark.parametrize("M,N,K", [(3072, 40, 102400), (384, 48, 8192), (256, 17, 4096 + 32 * 5)])
def test_gemm_f32_narrow_n(M, N, K):
    """N <= 48 exact NT GEMMs (layer 0's dW_ih = dG^T x at c2: M = 4H, N = 40, K = T B) on the
    narrow kernel (128 x 48 tiles of v_mfma_f32_16x16x4_f32, split-K slabs): against fp64, with a
    bias (the slab reduce's epilogue) on the ragged shape."""
    from pytorch_speaker_verification_amd.ops import gemm_f32
    g = torch.Generator().manual_seed(M + N + K)
    A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g) if N == 17 else None
    ref = A.double() @ B.double().T + (bias.double() if bias is not None else 0.0)
    C = gemm_f32(A.to(DEV), B.to(DEV), True, True, bias=bias.to(DEV) if bias is not None else None).cpu().double()
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    print(f"\nMEASURED gemm_f32_narrow.{M}x{N}x{K}.rel_vs_fp64 {err:.2e}")
    assert err <= 1e-5


@pytest.mark.parametrize("M,N,K", [(3072, 40, 102400), (384, 48, 8192), (256, 16, 4096 + 64)])
def test_gemm_bf16_narrow_n(M, N, K):
    """N <= 48 bf16 NT GEMMs (layer 0's dW_ih = dG^T x at c3: M = 4H, N = 40, K = T B) on the narrow
    kernel (128 x 48 tiles of v_mfma_f32_16x16x32_bf16, split-K slabs): against fp64 on the same
    bf16 operands, with a bias (the slab reduce's epilogue) on the smallest shape."""
    from pytorch_speaker_verification_amd._lib import call, lib, ptr
    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = torch.randn(M, K, generator=g).bfloat16()
    B = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g) if N == 16 else None
    ref = A.double() @ B.double().T + (bias.double() if bias is not None else 0.0)
    Ad, Bd = A.to(DEV), B.to(DEV)
    bd = bias.to(DEV) if bias is not None else None
    C = torch.full((M, N), float("nan"), device=DEV)
    ws = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=DEV)
    call("sv_gemm_bf16", M, N, K, ptr(Ad), K, ptr(Bd), K, ptr(C), N, ptr(bd) if bd is not None else None, None, 0.0,
         ptr(ws), torch.cuda.current_stream().cuda_stream)
    err = (C.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
    print(f"\nMEASURED gemm_bf16_narrow.{M}x{N}x{K}.rel_vs_fp64 {err:.2e}")
    assert err <= 1e-5


@pytest.mark.parametrize("M,N,K", [(9216, 2048, 96), (9216, 2048, 64), (16640, 1024, 32), (10240, 3072, 768)])
def test_gemm_f32_persistent_tiles_two_biases(M, N, K):
    """More 256 x 256 tiles than CUs: the persistent form (gemm_f32_256p_kernel: the next tile's
    k-tile 0 DMA'd during this tile's last k-tile), both bias vectors as K1 passes them; nk = 2 and
    nk = 1 (the one-shot kernel) included."""
    from pytorch_speaker_verification_amd._lib import call, ptr
    g = torch.Generator().manual_seed(M + N + K)
    A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    b0, b1 = torch.randn(N, generator=g), torch.randn(N, generator=g)
    Ad, Bd, b0d, b1d = A.to(DEV), B.to(DEV), b0.to(DEV), b1.to(DEV)
    C = torch.full((M, N), float("nan"), device=DEV)
    call("sv_gemm_f32", 1, 1, M, N, K, ptr(Ad), K, ptr(Bd), K, ptr(C), N, ptr(b0d), ptr(b1d), 0.0, None, 0,
         torch.cuda.current_stream().cuda_stream)
    ref = A.double() @ B.double().T + b0.double() + b1.double()
    err = (C.cpu().double() - ref).abs().max().item()
    assert err <= 2e-6 * K ** 0.5 * ref.abs().max().item() + 1e-5, err
    # repeatable bit for bit (the counted wait orders every tile's first k-tile)
    C2 = torch.full_like(C, float("nan"))
    call("sv_gemm_f32", 1, 1, M, N, K, ptr(Ad), K, ptr(Bd), K, ptr(C2), N, ptr(b0d), ptr(b1d), 0.0, None, 0,
         torch.cuda.current_stream().cuda_stream)
    assert torch.equal(C, C2)


@pytest.mark.parametrize("M,N,K", [(9216, 2048, 64), (5120, 3072, 768), (10240, 3072, 768)])
def test_gemm_bf16_bfout_two_biases(M, N, K):
    """The bf16-output K1 (persistent gemm_bf16_8qp_kernel, bias sums staged in LDS) is the RNE
    rounding of the fp32-output kernel's sums (same k-loop, same bias order) bit for bit."""
    from pytorch_speaker_verification_amd._lib import call, lib, ptr
    g = torch.Generator().manual_seed(M + 5 * N + K)
    A = torch.randn(M, K, generator=g).bfloat16().to(DEV)
    B = torch.randn(N, K, generator=g).bfloat16().to(DEV)
    b0, b1 = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    s = torch.cuda.current_stream().cuda_stream
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    call("sv_gemm_bf16_bf", M, N, K, ptr(A), K, ptr(B), K, ptr(Cb), N, ptr(b0), ptr(b1), s)
    C = torch.empty(M, N, device=DEV)
    ws = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=DEV)
    call("sv_gemm_bf16", M, N, K, ptr(A), K, ptr(B), K, ptr(C), N, ptr(b0), ptr(b1), 0.0, ptr(ws), s)
    assert torch.equal(Cb, C.bfloat16())
    ref = A.double() @ B.double().T + b0.double() + b1.double()
    assert (C.double() - ref).abs().max().item() <= 2e-6 * K ** 0.5 * ref.abs().max().item() + 1e-5


@pytest.mark.parametrize("M,N,K", [(640, 3072, 768), (3072, 768, 10240), (100, 40, 72), (640, 256, 768),
                                   (1024, 768, 3072), (2560, 3072, 768), (512, 256, 4096)])
def test_gemm_bf16(M, N, K):
    """bf16 operands, fp32 accumulation: against fp64 on the same bf16-rounded inputs."""
    from pytorch_speaker_verification_amd._lib import call, lib, ptr
    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = torch.randn(M, K, generator=g).bfloat16()
    B = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g)
    ref = A.double() @ B.double().T + bias.double()
    Ad, Bd, biasd = A.to(DEV), B.to(DEV), bias.to(DEV)
    C = torch.empty(M, N, device=DEV)
    ws = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=DEV)
    call("sv_gemm_bf16", M, N, K, ptr(Ad), K, ptr(Bd), K, ptr(C), N, ptr(biasd), None, 0.0, ptr(ws),
         torch.cuda.current_stream().cuda_stream)
    err = (C.cpu().double() - ref).abs().max().item()
    assert err <= 2e-6 * K ** 0.5 * ref.abs().max().item() + 1e-5, err


def test_f32_products_bf16x6_accuracy_and_step():
    """The opt-in bf16x6 fp32-product mode: GEMM error against fp64 no larger than the exact
    fp32-MFMA path's (x1.25 margin), and a full training step that agrees with the exact path
    to fp32 level (loss 1e-5 relative, parameters 1e-5 relative)."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    from pytorch_speaker_verification_amd.ops import F32_PRODUCT_MODES
    g = np.random.default_rng(3)
    M, N, K = 256, 512, 768
    A = g.standard_normal((M, K)).astype(np.float32)
    B = g.standard_normal((N, K)).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64).T
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64).T
    errs = {}
    for mode in ("mfma_f32", "bf16x6"):
        C = torch.empty(M, N, device=DEV)
        call("sv_gemm_f32", 1, 1, M, N, K, ptr(torch.tensor(A, device=DEV)), K, ptr(torch.tensor(B, device=DEV)),
             K, ptr(C), N, None, None, 0.0, None, F32_PRODUCT_MODES[mode], stream_of(C))
        errs[mode] = float((np.abs(C.cpu().numpy() - ref) / scale).max())
    assert errs["bf16x6"] <= 1.25 * errs["mfma_f32"], errs
    assert errs["bf16x6"] < 1e-6, errs

    from conftest import model_dims
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    dims, Ns, Ms, T = (40, 128, 3, 64), 6, 4, 20
    sd = recipe.make_weights(77, *dims, scale=3.0)
    x = torch.tensor(recipe.make_frames(78, Ns * Ms, T, dims[0]), device=DEV)
    res = {}
    for mode in ("mfma_f32", "bf16x6"):
        with model_dims(*dims):
            net = SpeechEmbedder()
        with torch.no_grad():
            for k, v in net.state_dict().items():
                v.copy_(torch.as_tensor(sd[k]))
        net = net.to(DEV)
        net.f32_products = mode  # a per-module setting, passed to the C ABI per call
        tr = GE2ETrainer(net, GE2ELoss(DEV), lr=0.01)
        loss = float(tr.step(x, Ns, Ms))
        res[mode] = (loss, tr.flat_p.detach().cpu().numpy().copy())
    (l0, p0), (l1, p1) = res["mfma_f32"], res["bf16x6"]
    assert abs(l1 - l0) <= 1e-5 * abs(l0), (l0, l1)
    assert np.abs(p1 - p0).max() <= 1e-5 * np.abs(p0).max()


@pytest.mark.parametrize("tag", ["n8m10_wb", "n4m5", "n3m2"])
@pytest.mark.parametrize("where", ["cuda", "cpu"])
def test_dropin_helpers_compose_and_train(tag, where):
    """GE2E composed from the re-exported drop-in helpers exactly as GE2ELoss.forward does
    (speech_embedder_net.py:45-48: centroids -> cossim -> w*cos+b -> calc_loss) and
    differentiated by autograd through the helpers' HIP backward kernels (sv_ge2e_*_bwd) matches
    the reference-generated golden dE / dw / db; 'cpu': the CPU-resident round trip."""
    from pytorch_speaker_verification_amd import speech_embedder_net as sen
    g = golden(f"ge2e_{tag}.npz")
    E0 = recipe.make_embeddings(int(g["seed"]), int(g["n"]), int(g["m"]), int(g["d"]), bool(g["clustered"]))
    E = torch.tensor(E0, device=where, requires_grad=True)
    w = torch.tensor(float(g["w"]), device=where, requires_grad=True)
    b = torch.tensor(float(g["b"]), device=where, requires_grad=True)
    centroids = sen.get_centroids(E)
    cossim = sen.get_cossim(E, centroids)
    sim_matrix = w * cossim + b
    loss, per = sen.calc_loss(sim_matrix)
    loss.backward()
    ref_loss = float(g["loss"])
    assert abs(float(loss) - ref_loss) <= 1e-4 * abs(ref_loss)
    np.testing.assert_allclose(per.detach().cpu().numpy(), g["per"], atol=1e-4)
    dE = E.grad.cpu().numpy()
    scale = np.abs(g["dE"]).max()
    err = float(np.abs(dE - g["dE"]).max() / scale)
    print(f"\nMEASURED helpers_autograd.{tag}.{where}.dE_rel {err:.3e}")
    assert err <= 1e-4, err
    assert abs(float(w.grad) - float(g["dw"])) <= 1e-4 * max(1.0, abs(float(g["dw"])))
    assert abs(float(b.grad) - float(g["db"])) <= 1e-4 * max(1.0, abs(float(g["db"])))


def test_dropin_calc_loss_per_embedding_gradient():
    """calc_loss's second output is differentiable too (a loss on per-embedding values):
    against torch autograd of the reference formula (utils.py:126-132) on the same S."""
    from pytorch_speaker_verification_amd.utils import calc_loss
    gen = torch.Generator().manual_seed(3)
    S = (torch.randn(5, 4, 7, generator=gen) * 3).double()
    wts = torch.randn(5, 4, generator=gen).double()
    Sr = S.clone().requires_grad_(True)
    idx = list(range(5))
    pos = Sr[idx, :, idx]
    neg = (torch.exp(Sr).sum(dim=2) + 1e-6).log()
    per_r = -(pos - neg)
    (per_r.sum() + (per_r * wts).sum()).backward()
    Sg = S.float().to(DEV).requires_grad_(True)
    loss, per = calc_loss(Sg)
    (loss + (per * wts.float().to(DEV)).sum()).backward()
    np.testing.assert_allclose(Sg.grad.cpu().numpy(), Sr.grad.numpy(), atol=2e-5)


@pytest.mark.parametrize("counts,offset", [((4096, 123, 8, 1, 3072 * 40), 0),             # scalar path (odd counts)
                                           ((640 * 160 * 40, 3072 * 40, 3072 * 768), 0),  # the bf16 forward's casts
                                           ((3072 * 768, 4096), 1)])                      # misaligned base: scalar
def test_cast_bf16_batch_is_rne(counts, offset):
    """sv_cast_bf16_batch (and sv_cast_bf16, a batch of one) = torch's round-to-nearest-even bf16
    cast, bit for bit, on the vectorised and the element-wise paths."""
    import ctypes
    from pytorch_speaker_verification_amd._lib import call, ptr
    g = torch.Generator().manual_seed(sum(counts))
    xs = [(torch.randn(n + offset, generator=g) * 3.0).to(DEV)[offset:] for n in counts]
    xs[0][:4] = torch.tensor([float("inf"), -0.0, 1.2e-38, 3.3895314e38])  # inf, signed zero, near min, bf16 max
    ys = [torch.empty(n, dtype=torch.bfloat16, device=DEV) for n in counts]
    n = len(xs)
    s = torch.cuda.current_stream().cuda_stream
    call("sv_cast_bf16_batch", n, (ctypes.c_void_p * n)(*[ptr(t) for t in xs]),
         (ctypes.c_void_p * n)(*[ptr(t) for t in ys]), (ctypes.c_long * n)(*[t.numel() for t in xs]), s)
    one = torch.empty(counts[-1], dtype=torch.bfloat16, device=DEV)
    call("sv_cast_bf16", ptr(xs[-1]), ptr(one), counts[-1], s)
    torch.cuda.synchronize()
    for x, y in zip(xs, ys):
        assert torch.equal(y.view(torch.int16), x.bfloat16().view(torch.int16))
    assert torch.equal(one.view(torch.int16), xs[-1].bfloat16().view(torch.int16))


@pytest.mark.parametrize("R,C,lds,ldd", [(3072, 768, 768, 3072), (3072, 40, 40, 3072), (40, 102400, 102400, 40),
                                         (100, 77, 80, 104), (3, 5, 5, 3)])
def test_transpose_cast_bf16(R, C, lds, ldd):
    """sv_transpose_cast_bf16 (the batched 64 x 64 tile kernel, one matrix): dst[c ldd + r] =
    bf16(src[r lds + c]) bit for bit, full and edge tiles, the 16-B and the element-wise paths."""
    from pytorch_speaker_verification_amd._lib import call, ptr
    g = torch.Generator().manual_seed(R * 31 + C)
    src = torch.randn(R, lds, generator=g).to(DEV)
    dst = torch.full((C, ldd), -7.0, dtype=torch.bfloat16, device=DEV)
    call("sv_transpose_cast_bf16", ptr(src), lds, R, C, ptr(dst), ldd, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = src[:, :C].t().bfloat16()
    assert torch.equal(dst[:, :R].view(torch.int16), ref.view(torch.int16))
    if ldd > R:  # padding columns untouched
        assert bool((dst[:, R:].float() == -7.0).all())


@pytest.mark.parametrize("N,M,D", [(160, 4, 64), (200, 3, 100), (129, 5, 256)])
def test_ge2e_fused_train_wide_n_other_d(N, M, D):
    """128 < N <= 256 with D != 256 takes the two-tile ge2e_rows_kernel<4> (D = 256 takes the
    register-blocked ge2e_rows4r_kernel, which the n256m10 golden covers): loss, per-row loss,
    dE, dw, db against the fp64 numpy oracle (oracle/ge2e_np.py, pinned to the reference's GE2E
    goldens by tests/test_oracle_golden.py).  Ragged N (129, 200: rows past the batch in the last
    tile) and D not a multiple of 64 (100)."""
    from pytorch_speaker_verification_amd import ops
    E = recipe.make_embeddings(N * 31 + D, N, M, D, True)
    w, b = 7.0, -3.0
    o_loss, o_per = ge2e_np.ge2e_forward(E, w, b)[:2]
    o_dE, o_dw, o_db = ge2e_np.ge2e_backward(E, w, b)
    Et = torch.tensor(E, device=DEV)
    wt = torch.tensor(w, dtype=torch.float32, device=DEV)
    bt = torch.tensor(b, dtype=torch.float32, device=DEV)
    loss, per, dE, dwdb = ops.ge2e_train(Et, wt, bt)
    loss, per, dE, dwdb = float(loss), per.cpu().numpy(), dE.cpu().numpy(), dwdb.cpu().numpy()
    scale = float(np.abs(o_dE).max())
    d_loss = abs(loss - float(o_loss)) / abs(float(o_loss))
    d_dE = float(np.abs(dE - o_dE).max()) / scale
    print(f"\nMEASURED ge2e_fused_wide.N{N}M{M}D{D} loss_rel {d_loss:.2e} dE_rel {d_dE:.2e} "
          f"dw {abs(dwdb[0] - o_dw):.2e} db {abs(dwdb[1] - o_db):.2e}")
    assert d_loss <= 1e-4
    np.testing.assert_allclose(per, o_per, atol=1e-4)
    assert d_dE <= 1e-4
    assert abs(dwdb[0] - o_dw) <= 1e-4 * max(1.0, abs(o_dw))
    assert abs(dwdb[1] - o_db) <= 1e-5 * N * M
