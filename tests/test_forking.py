"""utils.forking.fork_safe: a forked child never runs the finalizers of the parent's objects
through its cyclic garbage collector (those may own GPU resources of the parent's HIP runtime)."""
import gc
import multiprocessing as mp
import os

from textsummarization_on_flink_amd.utils.forking import fork_safe


class _Owner:
    """Stands in for a GPU-owning object: records which process finalised it."""

    def __init__(self, path):
        self.path = path
        self.me = self  # a reference cycle: only the cyclic collector frees it

    def __del__(self):
        with open(self.path, "a") as f:
            f.write(f"{os.getpid()}\n")


_HOLD = []


def _child():
    _HOLD.clear()  # the parent's cycle becomes garbage in the child ...
    gc.collect()   # ... and must not be finalised here
    os._exit(0)


def test_child_does_not_finalise_parent_cycles(tmp_path):
    path = str(tmp_path / "finalised")
    _HOLD.append(_Owner(path))
    ctx = mp.get_context("fork")
    with fork_safe():
        p = ctx.Process(target=_child)
        p.start()
    p.join(timeout=30)
    assert p.exitcode == 0
    assert not os.path.exists(path), open(path).read()
    _HOLD.clear()
    gc.collect()  # the parent still collects it
    assert open(path).read().split() == [str(os.getpid())]
