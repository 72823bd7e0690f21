"""utils.graphs.capture_guard: the cyclic collector runs before a capture sequence and stays off
inside it (a collection mid-capture can run HIP-calling destructors of unreachable engines)."""
import gc

from textsummarization_on_flink_amd.utils.graphs import capture_guard


class _Cyc:
    freed = 0

    def __init__(self):
        self.me = self

    def __del__(self):
        _Cyc.freed += 1


def test_capture_guard_collects_first_and_pauses_the_collector():
    gc.enable()
    _Cyc.freed = 0
    _Cyc()  # unreachable cycle
    with capture_guard():
        assert _Cyc.freed == 1          # collected before the capture
        assert not gc.isenabled()
        _Cyc()
        assert _Cyc.freed == 1          # nothing collected inside (automatic collection is off)
    assert gc.isenabled()
    gc.collect()
    assert _Cyc.freed == 2


def test_trainer_phase_object_holds_no_strong_reference():
    """GraphTrainer's phase-0 object refers to its trainer weakly: a dropped trainer (and its
    graphs) is freed by reference counting, not by a later cyclic collection."""
    import weakref

    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    class T:
        pass

    t = T()
    ph = GraphTrainer._Phase0(t)
    r = weakref.ref(t)
    del t
    assert r() is None and ph is not None
