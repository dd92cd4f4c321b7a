"""The single-input C-ABI forms named in SURVEY §8b (hgnn_linear_{fwd,dgrad,wgrad}_f32,
hgnn_hetero_epilogue[_bwd]) called through ctypes exactly as INTEGRATION.md §3 shows, against
plain torch fp32 (float64 for the reference values)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _lib():
    from truth_recommendation_gnn_amd import _native as N
    return N


def _close(got, ref):
    scale = float(ref.abs().max()) if ref.numel() else 0.0
    torch.testing.assert_close(got.double().cpu(), ref.cpu(), rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.parametrize("n,k,h", [(1000, 64, 64), (3000, 128, 64), (517, 37, 20), (0, 64, 64),
                                   (2048, 256, 128)])
def test_linear_single_forms(n, k, h):
    N = _lib()
    lib, p, st = N.lib(), N.ptr, N.stream_ptr(DEV)
    g = torch.Generator(device="cpu").manual_seed(n + k + h)
    x = torch.randn(n, k, generator=g).to(DEV)
    w = torch.randn(h, k, generator=g).to(DEV) / k ** 0.5
    b = torch.randn(h, generator=g).to(DEV)
    dy = torch.randn(n, h, generator=g).to(DEV)
    out = torch.empty(n, h, device=DEV)
    N.check(lib.hgnn_linear_fwd_f32(p(x), n, k, p(w), h, p(b), p(out), st), "fwd")
    _close(out, x.double() @ w.double().T + b.double())
    N.check(lib.hgnn_linear_fwd_f32(p(x), n, k, p(w), h, None, p(out), st), "fwd no bias")
    _close(out, x.double() @ w.double().T)
    dx = torch.empty(n, k, device=DEV)
    N.check(lib.hgnn_linear_dgrad_f32(p(dy), n, h, p(w), k, p(dx), st), "dgrad")
    _close(dx, dy.double() @ w.double())
    dw, db = torch.empty(h, k, device=DEV), torch.empty(h, device=DEV)
    ws = N.workspace(lib.hgnn_linear_bwd_ws_bytes(n, k, h), DEV)
    N.check(lib.hgnn_linear_wgrad_f32(p(x), p(dy), n, k, h, p(dw), p(db), p(ws), ws.numel(), st),
            "wgrad")
    _close(dw, dy.double().T @ x.double())
    _close(db, dy.double().sum(0))


@pytest.mark.parametrize("n_in,n,relu", [(2, 64 * 1000, 1), (3, 1001, 1), (1, 4096, 0),
                                         (6, 128 * 333, 1)])
def test_hetero_epilogue(n_in, n, relu):
    N = _lib()
    lib, p, st = N.lib(), N.ptr, N.stream_ptr(DEV)
    g = torch.Generator(device="cpu").manual_seed(n_in * n)
    ins = [torch.randn(n, generator=g).to(DEV) for _ in range(n_in)]
    wts = [1.0, 0.75, 0.5, 2.0, -1.0, 0.25][:n_in]
    out = torch.empty(n, device=DEV)
    warr = (ctypes.c_float * 6)(*wts)
    N.check(lib.hgnn_hetero_epilogue(n_in, N.ptr_array(ins), warr, n, relu, p(out), st), "epi")
    ref = sum(w * t.double() for w, t in zip(wts, ins))
    if relu:
        ref = ref.clamp_min(0)
    _close(out, ref)
    dout = torch.randn(n, generator=g).to(DEV)
    dins = [torch.empty(n, device=DEV) for _ in range(n_in)]
    dins[0] = None if n_in > 1 else dins[0]              # a skipped input gradient
    N.check(lib.hgnn_hetero_epilogue_bwd(n_in, warr, n, relu, p(out), p(dout),
                                         N.ptr_array(dins), st), "epi bwd")
    mask = (out > 0).double() if relu else torch.ones(n, dtype=torch.float64, device=DEV)
    for w, d in zip(wts, dins):
        if d is not None:
            _close(d, w * dout.double() * mask)


def test_single_forms_reject_bad_arguments():
    N = _lib()
    lib = N.lib()
    assert lib.hgnn_linear_dgrad_f32(None, 10, 4, None, 4, None, None) != 0
    assert lib.hgnn_linear_wgrad_f32(None, None, 10, 4, 4, None, None, None, 0, None) != 0
    assert lib.hgnn_hetero_epilogue(0, None, None, 10, 1, None, None) != 0
    assert b"epilogue" in lib.hgnn_last_error_string()
