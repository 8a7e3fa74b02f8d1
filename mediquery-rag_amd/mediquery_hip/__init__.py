"""mediquery_hip - MI355X-native dense-retrieval backend for MediQuery-RAG.

Drop-in replacements for the reference's retrieval pair:
    OllamaEmbeddings("shaw/dmeta-embedding-zh")  ->  HipBertEmbeddings
    langchain_chroma.Chroma                        ->  HipChroma
backed by libmqhip.so (hand-written HIP for gfx950, C ABI in include/mq.h).
"""
from .config import BertConfig, DMETA_BASE, GELU_ERF, GELU_TANH, POOL_CLS, POOL_MEAN
from .compat import Document, HAVE_LANGCHAIN
from ._lib import MQError, MQ_MAX_K, device_count, lib
from .native import Encoder, FlatIndex, merge_topk_device, merge_topk_host
from .embeddings import HipBertEmbeddings
from .vectorstore import HipChroma

# LangChain-compatible aliases for a one-line swap at src/medical_engine.py:25-26
OllamaEmbeddings = HipBertEmbeddings
Chroma = HipChroma

__all__ = ["BertConfig", "DMETA_BASE", "GELU_ERF", "GELU_TANH", "POOL_CLS", "POOL_MEAN",
           "Document", "HAVE_LANGCHAIN", "MQError", "MQ_MAX_K", "device_count", "lib", "Encoder",
           "FlatIndex", "merge_topk_device", "merge_topk_host", "HipBertEmbeddings", "HipChroma",
           "OllamaEmbeddings", "Chroma"]
