"""BertEmbedder with its encoder on the MI355X (mirror of the reference module).

Same class, arguments, results and errors as the reference's
``bert_embeddings.BertEmbedder`` (bert_embeddings.py:15-178): a tokenizer and
a ``transformers`` BERT loaded by name (:42-47), ``get_embedding`` /
``get_embeddings_batch`` with mean / cls / max pooling over
``last_hidden_state`` (:53-158, padding=True, truncation at max_length),
``compute_similarity`` (:160-178).

By default the forward pass is the reference's own: the torch model in fp32
on ``device`` (:46, :136). ``gpu_encoder=True`` moves it into libfheicp's
encoder on a GPU device (fheicp.bert.GpuBert): ``gpu_precision="f32"``
(default) keeps the reference's arithmetic on the f32 MFMA in another
summation order, ``"bf16"`` rounds the GEMM operands to bf16. Either way the
embeddings are not bit-equal to torch's, so ``provenance`` names the encoder
(None for torch) and batch_operations tags stored vectors with it and refuses
to score vectors of different encoders together.

``model=`` / ``tokenizer=`` take already-built objects (the weights and the
vocabulary are downloads the offline image does not have).
"""
from __future__ import annotations

import logging
from typing import List, Optional

import numpy as np

logger = logging.getLogger(__name__)

POOLINGS = ("mean", "cls", "max")


class BertEmbedder:
    """Extract BERT embeddings for text documents."""

    def __init__(self, model_name: str = 'bert-base-uncased', max_length: int = 100, device: Optional[str] = None,
                 model=None, tokenizer=None, gpu_encoder: bool = False, gpu_precision: str = 'f32'):
        import torch
        self.model_name = model_name
        self.max_length = min(max_length, 512)  # BERT's limit (:30)
        if device is None:
            self.device = 'cuda' if torch.cuda.is_available() else 'cpu'
        else:
            self.device = device
        logger.info(f"Using device: {self.device}")
        if tokenizer is None:
            from transformers import AutoTokenizer
            tokenizer = AutoTokenizer.from_pretrained(model_name)
        self.tokenizer = tokenizer
        if model is None:
            from transformers import AutoModel
            model = AutoModel.from_pretrained(model_name)
        self.model = model
        self.model.eval()
        self.hidden_size = self.model.config.hidden_size
        self.gpu = None
        if gpu_encoder:
            if not str(self.device).startswith('cuda'):
                raise ValueError("gpu_encoder=True needs a cuda device")
            from fheicp.bert import GpuBert
            idx = torch.device(self.device).index
            self.gpu = GpuBert(model=self.model, device=0 if idx is None else idx, precision=gpu_precision)
        else:
            self.model.to(self.device)
        logger.info(f"Model loaded. Hidden size: {self.hidden_size}")

    @property
    def provenance(self) -> Optional[str]:
        """None for the reference's torch forward, else the HIP encoder's tag."""
        return self.gpu.provenance if self.gpu is not None else None

    def _pooled(self, encoded, pooling: str) -> np.ndarray:
        if pooling not in POOLINGS:
            raise ValueError(f"Unknown pooling method: {pooling}")
        if self.gpu is not None:
            out = self.gpu.forward(encoded['input_ids'], encoded['attention_mask'], encoded.get('token_type_ids'),
                                   pooling=pooling)
            return out.cpu().numpy()
        import torch
        encoded = {k: v.to(self.device) for k, v in encoded.items()}
        with torch.no_grad():
            hidden_states = self.model(**encoded).last_hidden_state
        if pooling == 'mean':
            attention_mask = encoded['attention_mask'].unsqueeze(-1)
            emb = (hidden_states * attention_mask).sum(dim=1) / attention_mask.sum(dim=1)
        elif pooling == 'cls':
            emb = hidden_states[:, 0, :]
        else:
            emb = hidden_states.max(dim=1)[0]
        return emb.cpu().numpy()

    def get_embedding(self, text: str, pooling: str = 'mean') -> np.ndarray:
        """Numpy array of shape (hidden_size,) (bert_embeddings.py:53-101)."""
        encoded = self.tokenizer(text, padding=True, truncation=True, max_length=self.max_length,
                                 return_tensors='pt')
        return self._pooled(encoded, pooling)[0]

    def get_embeddings_batch(self, texts: List[str], batch_size: int = 8, pooling: str = 'mean') -> np.ndarray:
        """Numpy array of shape (n_texts, hidden_size), batch_size texts per
        forward pass (bert_embeddings.py:103-158)."""
        embeddings = []
        for i in range(0, len(texts), batch_size):
            encoded = self.tokenizer(texts[i:i + batch_size], padding=True, truncation=True,
                                     max_length=self.max_length, return_tensors='pt')
            embeddings.append(self._pooled(encoded, pooling))
        return np.vstack(embeddings)

    def compute_similarity(self, emb1: np.ndarray, emb2: np.ndarray) -> float:
        """Cosine similarity of two embeddings (bert_embeddings.py:160-178)."""
        emb1_norm = emb1 / np.linalg.norm(emb1)
        emb2_norm = emb2 / np.linalg.norm(emb2)
        return np.dot(emb1_norm, emb2_norm)
