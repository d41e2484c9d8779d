"""Graph-executable lifetime (utils/profiling.py, round 6): a dropped GraphedStep never calls HIP from its
finaliser -- the garbage collector can run it in the middle of another graph's capture or replay -- its executable
is parked and destroyed at exit (QDML_GRAPH_RELEASE=exit, the default) or at the next safe point (=sync: a device
sync outside any capture)."""
import gc

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.utils import profiling


class FakeGraph:
    def __init__(self, log):
        self.log = log

    def reset(self):
        self.log.append("reset")


def test_dropped_graph_is_parked_until_a_safe_point(monkeypatch):
    log = []
    profiling._GRAVEYARD.clear()
    monkeypatch.setattr(profiling, "GRAPH_RELEASE", "sync")
    gs = profiling.GraphedStep(lambda: None, enabled=False)
    gs.graph = FakeGraph(log)
    del gs
    gc.collect()
    assert log == [] and len(profiling._GRAVEYARD) == 1          # (the finaliser made no call)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: log.append("sync"))
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    profiling.release_dropped_graphs()
    assert log == [] and len(profiling._GRAVEYARD) == 1          # (a capture is running: not a safe point)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    profiling.release_dropped_graphs()
    assert log == ["sync", "reset"] and not profiling._GRAVEYARD


def test_close_releases_now_and_the_step_cannot_run_after(monkeypatch):
    log = []
    profiling._GRAVEYARD.clear()
    monkeypatch.setattr(profiling, "GRAPH_RELEASE", "sync")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: log.append("sync"))
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    gs = profiling.GraphedStep(lambda: None, enabled=False)
    gs.graph = FakeGraph(log)
    gs.close()
    assert log == ["sync", "reset"] and not profiling._GRAVEYARD
    try:
        gs()
    except RuntimeError as e:
        assert "after close" in str(e)
    else:
        raise AssertionError("a closed step ran")


def test_default_keeps_parked_graphs_until_exit(monkeypatch):
    """QDML_GRAPH_RELEASE=exit (default): close() and safe points leave the executable alone; the exit hook
    (release_dropped_graphs(final=True)) destroys it."""
    log = []
    profiling._GRAVEYARD.clear()
    monkeypatch.setattr(profiling, "GRAPH_RELEASE", "exit")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: log.append("sync"))
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    gs = profiling.GraphedStep(lambda: None, enabled=False)
    gs.graph = FakeGraph(log)
    gs.close()
    profiling.release_dropped_graphs()
    assert log == [] and len(profiling._GRAVEYARD) == 1
    profiling.release_dropped_graphs(final=True)
    assert log == ["sync", "reset"] and not profiling._GRAVEYARD
