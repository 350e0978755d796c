"""Host-side pieces of the target-function mirror (no GPU)."""
from gene2vec_amd import evaluate as EV


def test_gmt_quirks(tmp_path):
    g = tmp_path / "p.gmt"
    long = "\t".join(["L", "u"] + [f"G{i}" for i in range(51)]) + "\n"   # 53 fields: skipped
    ok = "\t".join(["P", "u", "A", "B", "C"]) + "\n"
    g.write_text(long + ok)
    pw = EV.read_pathways(str(g))
    assert pw == [ok]
    # the last field keeps its newline (reference quirk): "C\n" never matches "C"
    tmp = pw[0].split("\t")
    assert tmp[-1] == "C\n"


def test_gene_list_skips_header(tmp_path):
    f = tmp_path / "w.txt"
    f.write_text("2 3\nA 1 2 3\nB 4 5 6\n")
    assert EV.read_gene_list(str(f)) == ["A", "B"]
