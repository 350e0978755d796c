"""gene2vec_amd -- MI355X-native Gene2vec trainer.

The hot path (gensim 3.4 skip-gram negative sampling as driven by the
reference's src/gene2vec.py) runs in hand-written gfx950 kernels inside
``libg2v.so`` (C ABI: include/g2v.h), loaded with ctypes.  The Python layer
mirrors the reference interface:

    from gene2vec_amd import Word2Vec, KeyedVectors      # gensim.models.*
    from gene2vec_amd import generateMatrix              # src/generateMatrix.py
    python -m gene2vec_amd.gene2vec data_dir out_dir txt # src/gene2vec.py
"""
from .word2vec import KeyedVectors, Vocab, Word2Vec  # noqa: F401

__all__ = ["Word2Vec", "KeyedVectors", "Vocab"]
__version__ = "0.1.0"
