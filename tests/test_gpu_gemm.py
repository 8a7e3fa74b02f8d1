"""Unit tests of the MFMA GEMM core (gemm_f32.hpp) behind every encoder projection:
each tile geometry x epilogue on ragged shapes against a float64 torch reference
(|err| <= 2e-5 * sqrt(K) relative to the row/col norms), for the exact-f32 tiles (0-4),
the split-f32 tiles (5-7) and the 8-wave workgroup tiles (8-9)."""
import math

import numpy as np
import pytest

from mediquery_hip import _lib

pytestmark = pytest.mark.gpu


def _ref(A, W, b, R, epi):
    y = A.double() @ W.double().T + b.double()
    if epi == 1:
        y = 0.5 * y * (1 + torch_erf(y / math.sqrt(2)))
    elif epi == 2:
        y = 0.5 * y * (1 + (math.sqrt(2 / math.pi) * (y + 0.044715 * y ** 3)).tanh())
    elif epi == 3:
        y = y + R.double()
    return y


def torch_erf(x):
    import torch
    return torch.erf(x)


@pytest.mark.parametrize("tile", list(range(10)))
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(1, 768, 768), (77, 96, 64), (300, 2304, 768),
                                   (1000, 768, 3072), (4099, 200, 32), (32, 3072, 768), (256, 768, 3072)])
def test_gemm(require_gpu, tile, epi, M, N, K):
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    R = torch.randn(M, N, device=dev, generator=g)
    out = torch.full((M, N), float("nan"), device=dev)
    _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(b), _lib.ptr(R), _lib.ptr(out),
              M, N, K, epi, tile, _lib.stream_handle())
    torch.cuda.synchronize()
    ref = _ref(A, W, b, R, epi)
    err = (out.double() - ref).abs().max().item()
    assert not torch.isnan(out).any()
    assert err < 2e-5 * math.sqrt(K) * 4, err


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (300, 2304, 3072), (1024, 3072, 768)])
def test_split_f32_is_fp32_class(require_gpu, M, N, K):
    """The 3-way bf16 split with six MFMAs per product (tile 5) must be as accurate as
    the exact f32 MFMA (tile 0) against a float64 reference: max error within 3x."""
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.zeros(N, device=dev)
    ref = A.double() @ W.double().T
    errs = {}
    for tile in (0, 5):
        out = torch.empty(M, N, device=dev)
        _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(b), _lib.ptr(b), _lib.ptr(out),
                  M, N, K, 0, tile, _lib.stream_handle())
        torch.cuda.synchronize()
        errs[tile] = (out.double() - ref).abs().max().item()
    assert errs[5] <= 3 * errs[0] + 1e-7, errs

