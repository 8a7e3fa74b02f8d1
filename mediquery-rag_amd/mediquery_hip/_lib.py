"""ctypes binding of libmqhip.so (include/mq.h) - the reference-side FFI for this path.

The library is built in-tree by `make -C mediquery-rag_amd/csrc` (or
`__graft_entry__.build()`).  There is no CPU fallback: if the shared object is missing
or fails to load, importing the product classes raises immediately.
"""
import ctypes
import hashlib
import os

try:  # load torch's HIP runtime first so the process has exactly one libamdhip64
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for host-only use
    torch = None

LIB_PATH = os.environ.get("MQ_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "libmqhip.so")

MQ_OK = 0
MQ_DTYPE_F32, MQ_DTYPE_BF16, MQ_DTYPE_F32X6, MQ_DTYPE_F32_SCREEN = 0, 1, 2, 3
MQ_GELU_ERF, MQ_GELU_TANH = 0, 1
MQ_POOL_CLS, MQ_POOL_MEAN = 0, 1
MQ_MAX_K = 64
MQ_MASK_SET, MQ_MASK_AND, MQ_MASK_OR, MQ_MASK_CLEAR = 0, 1, 2, 3
# mq_encoder_set_option ids (include/mq.h)
MQ_ENC_OPT_ROWS_MAX, MQ_ENC_OPT_ROWS_SPLITS, MQ_ENC_OPT_SPLITK_MAX = 0, 1, 2
MQ_ENC_OPT_LN_ROWS_PER_WAVE, MQ_ENC_OPT_FUSE_ATTN_OPROJ, MQ_ENC_OPT_FUSED_LN = 3, 4, 5
MQ_ENC_OPT_SPLITK_TILES, MQ_ENC_OPT_LN_ON_LOAD, MQ_ENC_OPT_RESIDENT_LAYERS = 6, 7, 8
MQ_ENC_OPT_X6_PRESPLIT = 9
MQ_ENC_OPT_ROWS_PLANES = 10


class MQError(RuntimeError):
    """A libmqhip call returned a non-zero status."""

    def __init__(self, fn, code, msg):
        super().__init__("%s failed (status %d): %s" % (fn, code, msg))
        self.code = code


class BertConfigC(ctypes.Structure):
    _fields_ = [("vocab_size", ctypes.c_int), ("hidden", ctypes.c_int), ("layers", ctypes.c_int),
                ("heads", ctypes.c_int), ("ffn", ctypes.c_int), ("max_positions", ctypes.c_int),
                ("type_vocab", ctypes.c_int), ("ln_eps", ctypes.c_float), ("gelu", ctypes.c_int),
                ("pooling", ctypes.c_int)]

    @classmethod
    def from_config(cls, cfg):
        return cls(cfg.vocab_size, cfg.hidden, cfg.layers, cfg.heads, cfg.ffn, cfg.max_positions,
                   cfg.type_vocab, cfg.ln_eps, cfg.gelu, cfg.pooling)


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); every symbol include/mq.h declares
SIGNATURES = {
    "mq_last_error": (ctypes.c_char_p, []),
    "mq_version": (ctypes.c_char_p, []),
    "mq_build_source_hash": (ctypes.c_char_p, []),
    "mq_device_count": (_I, []),
    "mq_index_create": (_I, [_I, _I, _I64, _I, _PP]),
    "mq_index_destroy": (_I, [_P]),
    "mq_index_size": (_I, [_P, ctypes.POINTER(_I64)]),
    "mq_index_dim": (_I, [_P, ctypes.POINTER(_I)]),
    "mq_index_add": (_I, [_P, _P, _I64, _I, _P]),
    "mq_index_reset": (_I, [_P]),
    "mq_index_search": (_I, [_P, _P, _I64, _I, _P, _P, _I, _P]),
    "mq_index_get": (_I, [_P, _I64, _I64, _P, _I, _P]),
    "mq_index_select": (_I, [_P, _P, _I64, _P]),
    "mq_index_data": (_I, [_P, _PP]),
    "mq_index_set_precision": (_I, [_P, _I]),
    "mq_index_set_stream_threshold": (_I, [_P, _I]),
    "mq_index_set_threshold_scan": (_I, [_P, _I]),
    "mq_index_set_int8_screen": (_I, [_P, _I]),
    "mq_index_set_async_screen": (_I, [_P, _I]),
    "mq_index_rescans": (_I, [_P, _P, _P]),
    "mq_index_screen_fallbacks": (_I, [_P, _P, _P]),
    "mq_index_screen_skips": (_I, [_P, _P, _P]),
    "mq_index_set_timing": (_I, [_P, _I]),
    "mq_index_read_timing": (_I, [_P, _P, _I]),
    "mq_index_save": (_I, [_P, ctypes.c_char_p]),
    "mq_index_load": (_I, [_P, ctypes.c_char_p]),
    "mq_index_save_rows": (_I, [_P, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64]),
    "mq_index_load_append": (_I, [_P, ctypes.c_char_p]),
    "mq_mask_eval": (_I, [_P, _I64, _P, _I, _P, _I, _P]),
    "mq_mask_eval_bits": (_I, [_P, _I64, _P, _I, _P, _I, _P]),
    "mq_mask_combine": (_I, [_P, _P, _I64, _I, _P]),
    "mq_index_search_masked": (_I, [_P, _P, _I, _P, _P, _P, _I, _P]),
    "mq_index_search_masked_batch": (_I, [_P, _P, _I64, _I, _P, _P, _P, _I, _P]),
    "mq_index_masked_gathers": (_I, [_P, ctypes.POINTER(_I64)]),
    "mq_topk_merge_host": (_I, [_P, _P, _I, _I64, _I, _I, _P, _P]),
    "mq_topk_merge_device": (_I, [_P, _P, _I, _I64, _I, _I, _P, _P, _P]),
    "mq_encoder_create": (_I, [_I, ctypes.POINTER(BertConfigC), _PP]),
    "mq_encoder_destroy": (_I, [_P]),
    "mq_encoder_weight_count": (_I64, [ctypes.POINTER(BertConfigC)]),
    "mq_encoder_load_weights": (_I, [_P, _P, _I64]),
    "mq_encoder_set_precision": (_I, [_P, _I]),
    "mq_encoder_set_graphs": (_I, [_P, _I]),
    "mq_encoder_set_option": (_I, [_P, _I, _I]),
    "mq_encoder_get_option": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int)]),
    "mq_encoder_set_timing": (_I, [_P, _I]),
    "mq_encoder_read_timing": (_I, [_P, _P, _I]),
    "mq_encoder_embed": (_I, [_P, _P, _P, _I, _I, _P, _I, _P]),
    "mq_tokenizer_create_wordpiece": (_I, [ctypes.c_char_p, _I, _I, _PP]),
    "mq_tokenizer_create_wordpiece_tokens": (_I, [ctypes.POINTER(ctypes.c_char_p), _I, _I, _I, _PP]),
    "mq_tokenizer_create_char": (_I, [_I, _I, _PP]),
    "mq_tokenizer_destroy": (_I, [_P]),
    "mq_tokenizer_encode_batch": (_I, [_P, ctypes.POINTER(ctypes.c_char_p), _I, _I, _P, _P,
                                       ctypes.POINTER(_I)]),
    "mq_debug_gemm_f32": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "mq_debug_w3_bytes": (_I64, [_I, _I]),
    "mq_debug_split_w3": (_I, [_P, _I, _I, _P, _P]),
    "mq_debug_gemm_x6p": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "mq_debug_int8_screen": (_I, [_P, _P, _I, _P, _P, _P]),
}

_lib = None


def lib():
    """The loaded library; raises (never falls back) when it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libmqhip.so not found at %s - build it with "
                              "`make -C mediquery-rag_amd/csrc` or __graft_entry__.build()" % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH)
        # A/B runs of an older build (tools/ab_*.sh) may lack symbols added since: only
        # then (MQ_LIB_ALLOW_MISSING=1) are absent entry points left unbound
        allow_missing = os.environ.get("MQ_LIB_ALLOW_MISSING") == "1"
        for name, (res, args) in SIGNATURES.items():
            if allow_missing and not hasattr(h, name):
                continue
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def check(fn_name, rc):
    if rc != MQ_OK:
        raise MQError(fn_name, rc, lib().mq_last_error().decode("utf-8", "replace"))
    return rc


def call(fn_name, *args):
    return check(fn_name, getattr(lib(), fn_name)(*args))


CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
_STAMPED_EXT = (".hip", ".cpp", ".hpp", ".inc")


def tree_source_hash(csrc=CSRC):
    """csrc/Makefile's STAMPED hash recomputed from the sources beside the package: the
    sorted csrc/*.hip *.cpp *.hpp *.inc, then the Makefile, then include/mq.h."""
    names = sorted(f for f in os.listdir(csrc) if f.endswith(_STAMPED_EXT))
    paths = [os.path.join(csrc, f) for f in names]
    paths += [os.path.join(csrc, "Makefile"), os.path.join(csrc, "..", "..", "include", "mq.h")]
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def built_source_hash():
    """The source hash the loaded library was built from (mq_build_source_hash)."""
    return lib().mq_build_source_hash().decode()


def check_build_fresh():
    """Raise if the loaded library was not built from the sources in this tree (a stale
    prebuilt .so); a no-op when the sources are absent (an installed package)."""
    if not os.path.isdir(CSRC):
        return
    built, tree = built_source_hash(), tree_source_hash()
    if built != tree:
        raise ImportError("libmqhip.so at %s was built from sources %s, the tree holds %s: "
                          "rebuild with `make -C mediquery-rag_amd/csrc`" % (LIB_PATH, built, tree))


def device_count():
    return lib().mq_device_count()


def ptr(a):
    """Address of a numpy array / torch tensor / int as c_void_p."""
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(a.ctypes.data)


class device_scope:
    """`with device_scope(d):` makes cuda:d torch's current device (so stream_handle(None)
    is that device's current stream) - a no-op without torch / CUDA or for d None."""

    def __init__(self, device):
        self._ctx = None
        if device is not None and torch is not None and torch.cuda.is_available():
            self._ctx = torch.cuda.device(int(device))

    def __enter__(self):
        if self._ctx is not None:
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self._ctx is not None:
            return self._ctx.__exit__(*exc)
        return False


def stream_handle(stream=None):
    """hipStream_t of a torch stream (None -> torch's current stream on the device)."""
    if stream is None:
        if torch is None or not torch.cuda.is_available():
            return None
        stream = torch.cuda.current_stream()
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)
