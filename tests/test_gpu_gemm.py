"""Unit tests of the MFMA GEMM core (gemm_f32.hpp) behind every encoder projection:
each tile geometry x epilogue on ragged shapes against a float64 torch reference
(|err| <= 2e-5 * sqrt(K) relative to the row/col norms), for the exact-f32 tiles (0-4),
the split-f32 tiles with the split in the staging (5-7) and on pre-split P3 operands
(8-10, 11-13 with a P3 output), which must reproduce 5-7 bit for bit."""
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


@pytest.mark.parametrize("tile", list(range(8)))
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


def _bf16_rne(x):
    """float32 -> (bf16 bits as uint16, the bf16 value as float32), round to nearest even."""
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    return r.astype(np.uint16), (r.astype(np.uint32) << 16).view(np.float32)


def split_p3(x):
    """Host restatement of the P3 layout (gemm_f32.hpp split_chunk_p3): [R][K] float32 ->
    [R][K/16][3][16] bf16 bits, planes x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)."""
    R, K = x.shape
    planes = []
    rest = x.astype(np.float32)
    for _ in range(3):
        bits, val = _bf16_rne(rest)
        planes.append(bits)
        rest = (rest - val).astype(np.float32)
    return np.stack([p.reshape(R, K // 16, 16) for p in planes], axis=2)


def test_split_p3_is_exact():
    """Host check of the P3 restatement: the three planes sum back to x exactly."""
    x = np.random.default_rng(3).standard_normal((5, 64)).astype(np.float32) * 7
    p3 = split_p3(x)
    vals = (p3.astype(np.uint32) << 16).view(np.float32).astype(np.float64).sum(axis=2)
    np.testing.assert_array_equal(vals.reshape(5, 64), x.astype(np.float64))


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(77, 96, 64), (300, 2304, 768), (1000, 768, 3072), (513, 3072, 768)])
def test_p3_operands_bit_identical(require_gpu, epi, M, N, K):
    """Tiles 8-10 (P3 operands) equal tiles 5-7 (split in the staging) bit for bit, and
    tiles 11-13 write exactly split_p3 of that output."""
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + 3 * N + K)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    R = torch.randn(M, N, device=dev, generator=g)

    A3 = torch.empty(M, K * 3 // 2, device=dev)
    W3 = torch.empty(N, K * 3 // 2, device=dev)
    _lib.call("mq_debug_split_p3", _lib.ptr(A), K, M, K, _lib.ptr(A3), _lib.stream_handle())
    _lib.call("mq_debug_split_p3", _lib.ptr(W), K, N, K, _lib.ptr(W3), _lib.stream_handle())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(A3.cpu().numpy().view(np.uint16).reshape(M, K // 16, 3, 16),
                                  split_p3(A.cpu().numpy()))

    def run(tile, out):
        a, w = (A3, W3) if tile >= 8 else (A, W)
        _lib.call("mq_debug_gemm_f32", _lib.ptr(a), _lib.ptr(w), _lib.ptr(b), _lib.ptr(R), _lib.ptr(out),
                  M, N, K, epi, tile, _lib.stream_handle())
        torch.cuda.synchronize()
        return out.cpu().numpy()

    for t in range(3):
        ref = run(5 + t, torch.full((M, N), float("nan"), device=dev))
        got = run(8 + t, torch.full((M, N), float("nan"), device=dev))
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
        if epi != 3 and N % 16 == 0:
            p3 = run(11 + t, torch.zeros((M, N * 3 // 2), device=dev))
            np.testing.assert_array_equal(p3.view(np.uint16).reshape(M, N // 16, 3, 16), split_p3(ref))


def p3t_to_p3(buf, rows, K):
    """P3T buffer (uint16 view) -> P3 planes [rows][K/16][3][16] (pad rows dropped)."""
    rb = (rows + 31) // 32
    x = buf.reshape(rb, K // 16, 3, 2, 32, 8).transpose(0, 4, 1, 2, 3, 5)
    return x.reshape(rb * 32, K // 16, 3, 16)[:rows]


@pytest.mark.parametrize("epi", [0, 1, 3])
@pytest.mark.parametrize("M,N,K", [(77, 96, 64), (300, 2304, 768), (1000, 768, 3072), (513, 3072, 768),
                                   (8192, 768, 768)])
def test_wide_split_f32_bit_identical(require_gpu, epi, M, N, K):
    """The wide 8-wave kernel on P3T operands (tiles 14 / 15) equals the 4-wave split-f32
    tile (5) bit for bit; 16 / 17 write exactly the P3T split of that output."""
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + 5 * N + K)
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    R = torch.randn(M, N, device=dev, generator=g)
    pad = lambda r: (r + 31) // 32 * 32  # noqa: E731
    A3 = torch.empty(pad(M) * K * 3 // 2, device=dev)
    W3 = torch.empty(pad(N) * K * 3 // 2, device=dev)
    _lib.call("mq_debug_split_p3t", _lib.ptr(A), K, M, K, _lib.ptr(A3), _lib.stream_handle())
    _lib.call("mq_debug_split_p3t", _lib.ptr(W), K, N, K, _lib.ptr(W3), _lib.stream_handle())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(p3t_to_p3(A3.cpu().numpy().view(np.uint16), M, K), split_p3(A.cpu().numpy()))

    def run(tile, a, w, out):
        _lib.call("mq_debug_gemm_f32", _lib.ptr(a), _lib.ptr(w), _lib.ptr(b), _lib.ptr(R), _lib.ptr(out),
                  M, N, K, epi, tile, _lib.stream_handle())
        torch.cuda.synchronize()
        return out.cpu().numpy()

    ref = run(5, A, W, torch.full((M, N), float("nan"), device=dev))
    for tile in (14, 15):
        got = run(tile, A3, W3, torch.full((M, N), float("nan"), device=dev))
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
        if epi != 3 and N % 16 == 0:
            buf = run(tile + 2, A3, W3, torch.zeros(pad(M) * N * 3 // 2, device=dev))
            np.testing.assert_array_equal(p3t_to_p3(buf.view(np.uint16), M, N), split_p3(ref))
