"""Matrix .txt exporter -- mirror of the reference's src/generateMatrix.py:6-24.

``outputTxt(f)`` loads the model saved at ``f`` and writes ``f + ".txt"``:
one line per gene in ``wv.vocab`` order (first occurrence in the training
corpus), ``gene<TAB>`` followed by every float32 value as ``str(value) + " "``
and a newline -- the format GGIPNN_util.load_embedding_vectors,
tsne_multi_core.load_embedding and plot_gene2vec read with ``line.split()``.
"""
from __future__ import annotations

import numpy as np

from . import textio
from .word2vec import KeyedVectors


def load_embeddings(file_name):
    model = KeyedVectors.load(file_name)
    word_vector = model.wv
    vocabulary = list(word_vector.vocab.keys())
    idx = [word_vector.vocab[w].index for w in vocabulary]
    return np.asarray(word_vector.vectors[idx]), tuple(vocabulary)


def outputTxt(embeddings_file):
    wv, vocabulary = load_embeddings(embeddings_file)
    matrix_txt_file = embeddings_file + ".txt"
    # str(np.float32(v)) per value, formatted natively (gene2vec_amd.textio)
    text = textio.format_rows(wv.astype(np.float32), None, vocabulary, textio.TXT_MATRIX)
    with open(matrix_txt_file, "wb") as out:
        out.write(text)
    return matrix_txt_file
