"""GPU: the torch.library ops (library.py) run the same HIP kernels as the module path --
torch.library.opcheck (schema, fake implementation, autograd registration, AOT dispatch), the
library-dispatched modules against the default autograd.Function modules, and a torch.compile
(dynamo + AOT autograd, backend aot_eager: no code generation) training loss against eager."""
import numpy as np
import pytest
import torch

import recipe
from conftest import model_dims

pytestmark = pytest.mark.gpu
DEV = "cuda"
DIMS = (40, 64, 2, 32)


def _nets(precision):
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    sd = recipe.make_weights(91, *DIMS, scale=3.0)
    out = []
    for dispatch in ("function", "library"):
        with model_dims(*DIMS):
            net = SpeechEmbedder()
        with torch.no_grad():
            for k, v in net.state_dict().items():
                v.copy_(torch.as_tensor(sd[k]))
        net = net.to(DEV)
        net.precision, net.dispatch = precision, dispatch
        ge2e = GE2ELoss(DEV)
        ge2e.dispatch = dispatch
        out.append((net, ge2e))
    return out


def test_opcheck_sv_ops():
    from pytorch_speaker_verification_amd import library
    g = torch.Generator().manual_seed(3)
    x = torch.randn(12, 8, 40, generator=g).to(DEV).requires_grad_()
    sd = recipe.make_weights(5, *DIMS, scale=2.0)
    names = [f"LSTM_stack.{n}_l{l}" for l in range(DIMS[2]) for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    ps = [torch.tensor(sd[k], device=DEV).requires_grad_() for k in names + ["projection.weight", "projection.bias"]]
    for prec in ("f32", "bf16"):
        torch.library.opcheck(library.speech_embedder, (x, ps, prec, "auto"))
    E = torch.nn.functional.normalize(torch.randn(3, 4, 32, generator=g), dim=2).to(DEV).requires_grad_()
    w = torch.tensor(10.0, device=DEV, requires_grad=True)
    b = torch.tensor(-5.0, device=DEV, requires_grad=True)
    torch.library.opcheck(library.ge2e_loss, (E, w, b))


@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_library_dispatch_matches_function_dispatch(precision):
    (nf, gf), (nl, gl) = _nets(precision)
    x = torch.tensor(recipe.make_frames(92, 20, 24, 40), device=DEV)
    res = []
    for net, ge2e in ((nf, gf), (nl, gl)):
        emb = net(x)
        loss = ge2e(emb.view(4, 5, -1))
        loss.backward()
        res.append((emb.detach(), loss.detach(), {k: p.grad.detach().clone() for k, p in net.named_parameters()},
                    ge2e.w.grad.detach().clone()))
    (ef, lf, gf_, wf), (el, ll, gl_, wl) = res
    assert torch.equal(ef, el)            # the same forward kernels
    assert torch.equal(lf, ll)
    worst = max(float((gl_[k] - gf_[k]).abs().max() / gf_[k].abs().max().clamp_min(1e-30)) for k in gf_)
    print(f"\nMEASURED library_vs_function.{precision}.grad_rel {worst:.2e} dw {float((wl - wf).abs()):.2e}")
    assert worst <= 1e-6 and float((wl - wf).abs()) <= 1e-6 * max(1.0, float(wf.abs()))


def test_torch_compile_aot_eager_training_loss():
    from pytorch_speaker_verification_amd import library
    (nf, gf), _ = _nets("f32")
    params = nf.flat_params()
    x = torch.tensor(recipe.make_frames(93, 20, 24, 40), device=DEV)

    def loss_fn(x, w, b, *ps):
        emb = library.speech_embedder(x, list(ps), "f32", "auto")
        loss, _ = library.ge2e_loss(emb.view(4, 5, -1), w, b)
        return loss

    eager = loss_fn(x, gf.w, gf.b, *params)
    ge = torch.autograd.grad(eager, params)
    torch._dynamo.reset()
    compiled = torch.compile(loss_fn, backend="aot_eager", fullgraph=True)
    out = compiled(x, gf.w, gf.b, *params)
    gc = torch.autograd.grad(out, params)
    assert torch.equal(out.detach(), eager.detach())
    worst = max(float((a - c).abs().max() / a.abs().max().clamp_min(1e-30)) for a, c in zip(ge, gc))
    print(f"\nMEASURED library_compiled_vs_eager.grad_rel {worst:.2e}")
    assert worst <= 1e-6
