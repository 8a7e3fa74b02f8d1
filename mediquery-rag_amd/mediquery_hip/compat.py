"""LangChain interop: subclass the real base classes when langchain_core is
importable, otherwise provide duck-typed stand-ins with the same surface (the
reference's own environment has langchain_core; this image does not)."""
import asyncio

try:  # pragma: no cover - exercised only where langchain_core is installed
    from langchain_core.documents import Document  # type: ignore
    from langchain_core.embeddings import Embeddings as EmbeddingsBase  # type: ignore
    from langchain_core.vectorstores import VectorStore as VectorStoreBase  # type: ignore
    HAVE_LANGCHAIN = True
except Exception:
    HAVE_LANGCHAIN = False

    class Document:
        """Minimal langchain_core.documents.Document: page_content + metadata (+ id)."""

        def __init__(self, page_content, metadata=None, id=None, **kwargs):
            self.page_content = page_content
            self.metadata = dict(metadata or {})
            self.id = id
            self.type = "Document"

        def __eq__(self, other):
            return (isinstance(other, Document) and self.page_content == other.page_content
                    and self.metadata == other.metadata)

        def __repr__(self):
            return "Document(page_content=%r, metadata=%r)" % (self.page_content[:40], self.metadata)

    class EmbeddingsBase:
        def embed_documents(self, texts):
            raise NotImplementedError

        def embed_query(self, text):
            raise NotImplementedError

        async def aembed_documents(self, texts):
            return await asyncio.get_running_loop().run_in_executor(None, self.embed_documents, texts)

        async def aembed_query(self, text):
            return await asyncio.get_running_loop().run_in_executor(None, self.embed_query, text)

    class VectorStoreBase:
        def add_documents(self, documents, **kwargs):
            texts = [d.page_content for d in documents]
            metadatas = [d.metadata for d in documents]
            if "ids" not in kwargs:
                ids = [getattr(d, "id", None) for d in documents]
                if all(ids):
                    kwargs["ids"] = ids
            return self.add_texts(texts, metadatas, **kwargs)

        @classmethod
        def from_documents(cls, documents, embedding, **kwargs):
            texts = [d.page_content for d in documents]
            metadatas = [d.metadata for d in documents]
            return cls.from_texts(texts, embedding, metadatas=metadatas, **kwargs)

        def as_retriever(self, **kwargs):
            k = kwargs.get("search_kwargs", {}).get("k", 4)
            store = self

            class _Retriever:
                def invoke(self, query, **_):
                    return store.similarity_search(query, k=k)

                get_relevant_documents = invoke

            return _Retriever()
