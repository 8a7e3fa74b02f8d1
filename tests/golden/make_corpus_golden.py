"""Generate the parser golden fixture from the reference itself (run in the build
container only; the reference does not exist on the GPU box).

Imports `parse_custom_format` from /root/reference/src/ingest_medical.py:11-87 with
stub modules standing in for the three LangChain packages it imports at :3-5 (they are
not installed here; only `langchain_core.documents.Document` is used by the parser, as a
record with `.page_content` and `.metadata`).  Runs it on the reference corpus
data/medical_data.txt and writes:

  tests/golden/medical_data.txt   - the parser input (data file, copied verbatim)
  tests/golden/corpus_docs.json   - the 154 (page_content, metadata) records + sha256

Usage:  python tests/golden/make_corpus_golden.py [/root/reference]
"""
import hashlib
import json
import os
import shutil
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))


class _Document:  # stand-in for langchain_core.documents.Document
    def __init__(self, page_content, metadata=None):
        self.page_content = page_content
        self.metadata = dict(metadata or {})


def _install_stubs():
    lc_ollama = types.ModuleType("langchain_ollama")
    lc_ollama.OllamaEmbeddings = object
    lc_chroma = types.ModuleType("langchain_chroma")
    lc_chroma.Chroma = object
    lc_core = types.ModuleType("langchain_core")
    lc_docs = types.ModuleType("langchain_core.documents")
    lc_docs.Document = _Document
    lc_core.documents = lc_docs
    for name, mod in [("langchain_ollama", lc_ollama), ("langchain_chroma", lc_chroma),
                      ("langchain_core", lc_core), ("langchain_core.documents", lc_docs)]:
        sys.modules.setdefault(name, mod)


def main(ref_root="/root/reference"):
    _install_stubs()
    sys.dont_write_bytecode = True  # never write into the read-only reference tree
    sys.path.insert(0, os.path.join(ref_root, "src"))
    import ingest_medical  # noqa: E402  (reference module, parse only)

    src_txt = os.path.join(ref_root, "data", "medical_data.txt")
    docs = ingest_medical.parse_custom_format(src_txt)
    recs = [{"page_content": d.page_content, "metadata": d.metadata} for d in docs]
    digest = hashlib.sha256("\x00".join(r["page_content"] for r in recs).encode("utf-8")).hexdigest()
    shutil.copyfile(src_txt, os.path.join(HERE, "medical_data.txt"))
    with open(os.path.join(HERE, "corpus_docs.json"), "w", encoding="utf-8") as f:
        json.dump({"source": "reference src/ingest_medical.py:11-87 on data/medical_data.txt",
                   "count": len(recs), "sha256_page_content_nul_joined": digest,
                   "docs": recs}, f, ensure_ascii=False, indent=0)
    print(len(recs), digest)


if __name__ == "__main__":
    main(*sys.argv[1:])
