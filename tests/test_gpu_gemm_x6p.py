"""K2p, the pre-split split-f32 encoder GEMM (csrc/gemm_x6p.hip): the weight split once
into its W3 plane image, the activations split while their fragments are read.

* bit-identical to the split-f32 tiles of gemm_f32.hpp (mq_debug_gemm_f32 tile 5) on
  every tile shape, epilogue and ragged shape: same split, same six products, same order;
* within the GEMM tolerance of tests/test_gpu_gemm.py against a float64 reference;
* the W3 image itself against a numpy restatement of the exact 3-way split."""
import math

import numpy as np
import pytest

from mediquery_hip import _lib
from test_gpu_gemm import _ref

pytestmark = pytest.mark.gpu

SHAPES = [(1, 768, 768), (77, 96, 64), (300, 2304, 768), (1000, 768, 3072), (4099, 200, 32),
          (32, 3072, 768), (256, 768, 3072), (513, 1536, 768)]


def _split_w3(W):
    import torch
    N, K = W.shape
    w3 = torch.empty(_lib.lib().mq_debug_w3_bytes(N, K), dtype=torch.uint8, device=W.device)
    _lib.call("mq_debug_split_w3", _lib.ptr(W), N, K, _lib.ptr(w3), _lib.stream_handle())
    return w3


def _x6p(A, w3, b, R, M, N, K, epi, tile):
    import torch
    out = torch.full((M, N), float("nan"), device=A.device)
    _lib.call("mq_debug_gemm_x6p", _lib.ptr(A), _lib.ptr(w3), _lib.ptr(b), _lib.ptr(R), _lib.ptr(out),
              M, N, K, epi, tile, _lib.stream_handle())
    torch.cuda.synchronize()
    return out


def _operands(M, N, K, dev):
    import torch
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    R = torch.randn(M, N, device=dev, generator=g)
    return A, W, b, R


@pytest.mark.parametrize("tile", [-1, 0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_x6p_bit_identical_to_x6_tiles(require_gpu, tile, epi, M, N, K):
    import torch
    dev = torch.device("cuda", 0)
    A, W, b, R = _operands(M, N, K, dev)
    w3 = _split_w3(W)
    got = _x6p(A, w3, b, R, M, N, K, epi, tile)
    ref6 = torch.full((M, N), float("nan"), device=dev)
    _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(b), _lib.ptr(R), _lib.ptr(ref6),
              M, N, K, epi, 5, _lib.stream_handle())
    torch.cuda.synchronize()
    assert not torch.isnan(got).any()
    assert torch.equal(got, ref6), (got - ref6).abs().max().item()
    err = (got.double() - _ref(A, W, b, R, epi)).abs().max().item()
    assert err < 2e-5 * math.sqrt(K) * 4, err


def _split3_np(x):
    """Exact 3-way split of fp32 x into bf16 planes (round-to-nearest-even per plane)."""
    planes = []
    r = x.astype(np.float32)
    for _ in range(3):
        u = r.view(np.uint32).astype(np.uint64)
        rounded = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        planes.append(rounded)
        r = (r - (rounded.astype(np.uint32) << 16).view(np.float32)).astype(np.float32)
    return planes


@pytest.mark.parametrize("N,K", [(96, 64), (200, 32), (768, 768)])
def test_w3_image_layout(require_gpu, N, K):
    import torch
    dev = torch.device("cuda", 0)
    W = torch.randn(N, K, device=dev, generator=torch.Generator(device=dev).manual_seed(N + K))
    img = _split_w3(W).cpu().numpy().view(np.uint16)
    torch.cuda.synchronize()
    planes = _split3_np(W.cpu().numpy())
    np_ = (N + 31) // 32 * 32
    for p in range(3):
        full = np.zeros((np_, K), np.uint16)
        full[:N] = planes[p]
        # W3[nb][kb][p][h][r][j]: row 32 nb + r, k = 16 kb + 8 h + j
        want = full.reshape(np_ // 32, 32, K // 16, 2, 8).transpose(0, 2, 3, 1, 4)
        got = img.reshape(np_ // 32, K // 16, 3, 2, 32, 8)[:, :, p]
        assert np.array_equal(got, want), p
    # the planes sum back to W exactly (fp32 residual arithmetic is exact)
    rec = sum((planes[p].astype(np.uint32) << 16).view(np.float32).astype(np.float64) for p in range(3))
    assert np.max(np.abs(rec - W.cpu().numpy().astype(np.float64)) / (np.abs(W.cpu().numpy()) + 1e-30)) < 2 ** -23
