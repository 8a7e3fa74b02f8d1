"""Encoder oracle (explicit torch-CPU BERT) vs transformers.BertModel golden vectors
(tests/golden/make_encoder_golden.py), all on seeded synthetic weights."""
import json
import os

import numpy as np
import pytest

from mediquery_hip.config import BertConfig, DMETA_BASE, GELU_TANH, POOL_MEAN
from mediquery_hip.tokenizer import CharTokenizer
from mediquery_hip.weights import synthetic_state_dict
from oracle.encoder import OracleEncoder
from oracle.flat import check_topk, exact_scores

TOL = 2e-5  # fp32 CPU vs fp32 CPU, different summation order


@pytest.fixture(scope="module")
def enc_golden(golden):
    return np.load(os.path.join(golden, "encoder_golden.npz"))


@pytest.mark.parametrize("case,cfg", [
    ("tiny_a", BertConfig(layers=2)),
    ("tiny_b", BertConfig(layers=2)),
    ("tiny_b_mean", BertConfig(layers=2, pooling=POOL_MEAN)),
    ("tiny_tanh", BertConfig(layers=2, gelu=GELU_TANH)),
])
def test_oracle_matches_transformers(enc_golden, case, cfg):
    src = case.replace("_mean", "")
    enc = OracleEncoder(cfg, synthetic_state_dict(cfg, 0))
    got = enc.embed(enc_golden[src + "_ids"], enc_golden[src + "_mask"])
    np.testing.assert_allclose(got, enc_golden[case + "_emb"], atol=TOL, rtol=0)
    np.testing.assert_allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-6)


def test_oracle_base_model(enc_golden):
    enc = OracleEncoder(DMETA_BASE, synthetic_state_dict(DMETA_BASE, 0))
    got = enc.embed(enc_golden["base_ids"], enc_golden["base_mask"])
    np.testing.assert_allclose(got, enc_golden["base_emb"], atol=TOL, rtol=0)


def test_config1_golden_is_self_consistent(golden):
    """Top-5 of the committed config-1 embeddings equals the committed ids (checker)."""
    g = np.load(os.path.join(golden, "config1_golden.npz"))
    s = exact_scores(g["query_emb"], g["doc_emb"])
    assert check_topk(g["top5_ids"], g["top5_scores"], s, 5, tol=1e-9, score_tol=1e-9) == []


def test_char_tokenizer_deterministic():
    t = CharTokenizer()
    ids, mask = t(["血糖 高", "心"])
    assert ids.shape == (2, 5) and ids[0, 0] == 101 and ids[0, 4] == 102
    assert mask.tolist() == [[1, 1, 1, 1, 1], [1, 1, 1, 0, 0]]
    assert t.token_id("血") == t.token_id("血") and 106 <= t.token_id("血") < 21128
