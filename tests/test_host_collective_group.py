"""CPU: the host transport's collective group (distributed.host_collective).

Under an nccl default group (a GPU node) the host transport's CPU tensors
need a gloo group of their own; under gloo the default group serves.  The
process group is stubbed: no nccl on this container."""
import torch.distributed as dist

from gene2vec_amd import distributed as Dd


def test_gloo_group_under_nccl_default_group_otherwise(monkeypatch):
    made = []
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(dist, "new_group", lambda **kw: made.append(kw) or "gloo-group")
    assert Dd.host_collective().group == "gloo-group"
    assert made == [{"backend": "gloo"}]
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "gloo")
    assert Dd.host_collective().group is None
    assert Dd.host_collective("given").group == "given"
    assert len(made) == 1
