"""CPU oracle for the Gene2vec SGNS hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker / the timed
CPU baseline.  The product path (``gene2vec_amd``) never imports it: it runs
the HIP library ``libg2v.so`` and fails loudly when that library is missing.

Contents
--------
``sgns_oracle.py``  NumPy / pure-Python restatement of gensim 3.4.0's
                    ``Word2Vec(sg=1, negative=5, hs=0)`` training path as driven
                    by the reference's ``src/gene2vec.py:70,86-88``.
``sgns_oracle.c``   The same semantics in C (sequential "workers=1" order and a
                    Hogwild OpenMP variant used as the CPU baseline).
``Makefile``        Builds ``oracle/build/liboracle.so`` from ``sgns_oracle.c``.
``target_oracle.py`` ``src/evaluation_target_function.py`` restated (numpy).
``coexpr_oracle.py`` ``src/generate_gene_pairs.py:45-65`` (coexpr) through
                    pandas' own ``DataFrame.corr`` -- the reference's library,
                    importable here, so this path's parity IS pinned.

Parity status: **parity unpinned.**  The algorithm lives in gensim 3.4.0
(``gensim/models/word2vec_inner.pyx``, ``word2vec.py``, ``base_any2vec.py``),
a third-party dependency that is not vendored in ``/root/reference`` and is not
importable offline; the reference ships no tests and no golden vectors
(SURVEY.md section 4 / 8(c)).  The restatement is pinned only where an
independent anchor exists: the reference's own fixture ``data/test.txt``
(counts, vocabulary size), numpy's ``RandomState`` (the very generator gensim
calls for ``seeded_vector`` and ``model.random``), and the closed-form
known-answer values recorded in SURVEY.md section 4.
"""
