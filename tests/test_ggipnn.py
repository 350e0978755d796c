"""GGIPNN harness pieces (CPU): the reference's data-pipeline semantics and a
learnability sanity check of the PyTorch restatement."""
import numpy as np

from gene2vec_amd import ggipnn as G


def test_fit_dict_and_fit_semantics():
    lines = ["A B", "B C", "A B C", " D  E", "C D"]
    d = G.my_fit_dict(lines, 2)
    # " D  E".strip().split(" ") == ["D", "", "E"] -> not 2 fields -> skipped
    assert d == {"A": 0, "B": 1, "C": 2, "D": 3}
    x = G.my_fit(lines, 2, d)
    assert x.tolist() == [[0, 1], [1, 2], [1, 1], [1, 1], [2, 3]]
    assert G.one_hot(["1", "0"]).tolist() == [[0, 1], [1, 0]]


def test_embedding_loader(tmp_path):
    f = tmp_path / "e.txt"
    f.write_text("A\t1.0 2.0 \nZ\t9 9 \n")
    emb = G.load_embedding_vectors({"A": 0, "B": 1}, str(f), 2, np.random.RandomState(0))
    assert emb[0].tolist() == [1.0, 2.0]
    assert np.all(np.abs(emb[1]) <= 0.25)


def test_learns_a_separable_signal(tmp_path):
    rng = np.random.RandomState(1)
    genes = [f"G{i}" for i in range(200)]
    vec = rng.randn(200, 8).astype(np.float32)
    def split(n, name):
        a = rng.randint(0, 200, n)
        b = rng.randint(0, 200, n)
        lab = (vec[a, 0] + vec[b, 0] > 0).astype(int)
        (tmp_path / f"{name}_text.txt").write_text("\n".join(f"{genes[i]} {genes[j]}" for i, j in zip(a, b)))
        (tmp_path / f"{name}_label.txt").write_text("\n".join(map(str, lab)))
    split(20000, "train")
    split(500, "valid")
    split(2000, "test")
    emb = tmp_path / "emb.txt"
    emb.write_text("".join(g + "\t" + "".join(f"{v} " for v in vec[i]) + "\n" for i, g in enumerate(genes)))
    auc = G.train_and_auc(str(emb), str(tmp_path), seed=0, embedding_size=8, num_epochs=3)
    assert auc > 0.9
