"""Matrix .txt exporter -- mirror of the reference's src/generateMatrix.py:6-24.

``outputTxt(f)`` loads the model saved at ``f`` and writes ``f + ".txt"``:
one line per gene in ``wv.vocab`` order (first occurrence in the training
corpus), ``gene<TAB>`` followed by every float32 value as ``str(value) + " "``
and a newline -- the format GGIPNN_util.load_embedding_vectors,
tsne_multi_core.load_embedding and plot_gene2vec read with ``line.split()``.
"""
from __future__ import annotations

import numpy as np

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
    rows = wv.astype(np.float32).astype(str)  # == str(np.float32(v)) element-wise
    with open(matrix_txt_file, "w") as out:
        for word, vals in zip(vocabulary, rows):
            out.write(str(word) + "\t" + "".join(v + " " for v in vals) + "\n")
    return matrix_txt_file
