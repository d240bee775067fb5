"""CPU: the torch.library ops of library.py are registered with the dispatcher, their fake
implementations give the right output shapes on fake CUDA tensors (no GPU needed), and a whole
GE2E training loss with its backward traces through make_fx into single sv:: op nodes -- what
torch.compile / torch.export see of the hot path."""
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.proxy_tensor import make_fx

from pytorch_speaker_verification_amd import library  # noqa: F401  (registers the sv:: ops)

DIMS = (40, 64, 2, 32)  # nmels, hidden, layers, proj


def _params(dev):
    F, H, L, P = DIMS
    ps = []
    for l in range(L):
        ps += [torch.empty(4 * H, F if l == 0 else H, device=dev), torch.empty(4 * H, H, device=dev),
               torch.empty(4 * H, device=dev), torch.empty(4 * H, device=dev)]
    return ps + [torch.empty(P, H, device=dev), torch.empty(P, device=dev)]


def test_ops_registered_with_schemas():
    for name in ("speech_embedder", "speech_embedder_backward", "ge2e_loss", "ge2e_loss_backward"):
        op = getattr(torch.ops.sv, name).default
        assert op._schema.name == f"sv::{name}"
    s = str(torch.ops.sv.speech_embedder.default._schema)
    assert "Tensor x" in s and "Tensor[] params" in s and "str precision" in s


def test_fake_shapes_on_fake_cuda_tensors():
    with FakeTensorMode():
        x = torch.empty(12, 8, 40, device="cuda")
        ps = _params("cuda")
        emb = torch.ops.sv.speech_embedder(x, ps, "f32", "auto")
        assert emb.shape == (12, 32) and emb.device.type == "cuda" and emb.dtype == torch.float32
        out = torch.ops.sv.speech_embedder_backward(x, ps, emb, "bf16", "auto", True)
        assert [tuple(t.shape) for t in out] == [tuple(x.shape)] + [tuple(p.shape) for p in ps]
        out = torch.ops.sv.speech_embedder_backward(x, ps, emb, "f32", "auto", False)
        assert out[0].numel() == 0
        E = torch.empty(3, 4, 32, device="cuda")
        w, b = torch.empty((), device="cuda"), torch.empty((), device="cuda")
        loss, per = torch.ops.sv.ge2e_loss(E, w, b)
        assert loss.shape == () and per.shape == (3, 4)
        dE, dw, db = torch.ops.sv.ge2e_loss_backward(E, w, b, loss)
        assert dE.shape == E.shape and dw.shape == () and db.shape == ()


def test_training_loss_and_backward_trace_to_sv_ops():
    def step(x, w, b, *ps):
        emb = library.speech_embedder(x, list(ps), "f32", "auto")
        loss, _ = library.ge2e_loss(emb.view(3, 4, -1), w, b)
        return torch.autograd.grad(loss, [x, w, b, *ps])

    # (fake CPU tensors: the autograd engine needs a live device context for CUDA ones, and the
    # fake implementations do not depend on the device)
    with FakeTensorMode() as mode:
        x = torch.empty(12, 8, 40, requires_grad=True)
        w = torch.empty((), requires_grad=True)
        b = torch.empty((), requires_grad=True)
        ps = [p.requires_grad_() for p in _params("cpu")]
        gm = make_fx(step, tracing_mode="fake")(x, w, b, *ps)
    targets = [str(n.target) for n in gm.graph.nodes if n.op == "call_function"]
    for op in ("sv.speech_embedder.default", "sv.ge2e_loss.default", "sv.ge2e_loss_backward.default",
               "sv.speech_embedder_backward.default"):
        assert op in targets, (op, targets)
    del mode
