"""Seeded synthetic inputs for parity tests and benchmarks.

corpus:   N x dim standard normal rows (seed 20260215), or the clustered variant
          (4096 Gaussian centroids + sigma 0.35 noise) so neighbours are meaningful;
          the index L2-normalises rows on add.
queries:  B unit vectors (seed 7); the first half planted as corpus rows + sigma 0.05
          noise, so their top-1 row is known.
tokens:   [CLS]=101, L-2 ids ~ U[106, vocab), [SEP]=102; mask all ones.
"""
import numpy as np

CORPUS_SEED = 20260215
QUERY_SEED = 7
TOKEN_SEED = 1


def corpus(n, dim=768, seed=CORPUS_SEED, clustered=False, chunk=1 << 16):
    rng = np.random.default_rng(seed)
    out = np.empty((n, dim), dtype=np.float32)
    if clustered:
        cents = rng.standard_normal((4096, dim), dtype=np.float32)
        for s in range(0, n, chunk):
            m = min(chunk, n - s)
            out[s:s + m] = cents[rng.integers(0, 4096, m)] + 0.35 * rng.standard_normal((m, dim), dtype=np.float32)
    else:
        for s in range(0, n, chunk):
            m = min(chunk, n - s)
            out[s:s + m] = rng.standard_normal((m, dim), dtype=np.float32)
    return out


def queries(b, corpus_rows, seed=QUERY_SEED, planted_frac=0.5, noise=0.05):
    """-> (queries [b, dim] unit-norm f32, planted row id per query or -1)."""
    rng = np.random.default_rng(seed)
    n, dim = corpus_rows.shape
    q = rng.standard_normal((b, dim), dtype=np.float32)
    planted = np.full(b, -1, dtype=np.int64)
    n_pl = int(b * planted_frac)
    if n_pl and n:
        planted[:n_pl] = rng.integers(0, n, n_pl)
        base = corpus_rows[planted[:n_pl]].astype(np.float32)
        base /= np.maximum(np.linalg.norm(base, axis=1, keepdims=True), 1e-12)
        q[:n_pl] = base + noise * q[:n_pl] / np.sqrt(dim)
    q /= np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-12)
    return q, planted


def token_batch(b, seq_len, vocab=21128, seed=TOKEN_SEED):
    rng = np.random.default_rng(seed)
    ids = rng.integers(106, vocab, size=(b, seq_len), dtype=np.int32)
    ids[:, 0] = 101
    ids[:, -1] = 102
    return ids, np.ones((b, seq_len), dtype=np.int32)


def corpus_device(n, dim, device, seed=CORPUS_SEED):
    """Large corpora generated directly in HBM (torch Philox RNG; seeded, but not the
    same values as `corpus`): used where parity is checked through planted queries."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randn((n, dim), generator=g, device=device, dtype=torch.float32)


# exact duplicate rows of the reference corpus: data/medical_data.txt parses to 154 docs
# whose page_content repeats at rows (72, 74), (104, 105), (110, 111), (120, 121) (SURVEY.md
# §8c); the clustered device corpus repeats that pattern in every block of 154 rows
REF_DUPLICATE_PAIRS = ((72, 74), (104, 105), (110, 111), (120, 121))


def clustered_corpus_device(n, dim, device, seed=CORPUS_SEED, n_centroids=4096, sigma=0.35,
                            duplicates=True):
    """SURVEY.md §8d's clustered variant generated in HBM: rows = one of `n_centroids`
    standard-normal centroids + sigma noise (cluster-mates at cosine ~0.89), plus the
    reference corpus's exact-duplicate pattern.  -> (rows [n, dim], centroid id per row)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    cents = torch.randn((n_centroids, dim), generator=g, device=device)
    assign = torch.randint(0, n_centroids, (n,), generator=g, device=device)
    rows = torch.randn((n, dim), generator=g, device=device)
    rows.mul_(sigma).add_(cents[assign])
    if duplicates and n >= 154:
        base = torch.arange(0, n - 153, 154, device=device)
        for a, b in REF_DUPLICATE_PAIRS:
            rows[base + b] = rows[base + a]
            assign[base + b] = assign[base + a]
    return rows, assign


def corpus_shard_device(rows_per_shard, shard, dim, device, seed=CORPUS_SEED):
    """Shard `shard` of a corpus made of equal seeded blocks (BASELINE config 4: 10M rows
    as 8 x 1.25M): every rank regenerates only the blocks it owns, and the global corpus
    is the same whatever the number of ranks."""
    return corpus_device(rows_per_shard, dim, device, seed=seed + 1 + shard)


def queries_device(b, rows_dev, seed=QUERY_SEED, planted_frac=0.5, noise=0.05):
    """Device twin of `queries` for corpora made by corpus_device."""
    import torch
    dev = rows_dev.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    n, dim = rows_dev.shape
    q = torch.randn((b, dim), generator=g, device=dev)
    planted = torch.full((b,), -1, dtype=torch.int64, device=dev)
    n_pl = int(b * planted_frac)
    if n_pl:
        planted[:n_pl] = torch.randint(0, n, (n_pl,), generator=g, device=dev)
        base = torch.nn.functional.normalize(rows_dev[planted[:n_pl]], dim=1)
        q[:n_pl] = base + noise * q[:n_pl] / dim ** 0.5
    return torch.nn.functional.normalize(q, dim=1), planted
