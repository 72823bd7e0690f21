"""Forking worker processes from a process that may already hold GPU state.

The data-loader workers (``data/loader.py``) and the stream packers (``data/stream_pack.py``)
are forked without exec and never touch the GPU. A forked child still inherits the parent's
heap, including uncollected reference cycles that own HIP resources (tensors, streams, graphs
of earlier work in the same process, e.g. a GPU test session). If the child's cyclic garbage
collector frees such a cycle, its destructors call into the HIP runtime of a process that
never initialised it, and the child crashes (seen as SIGSEGV inside ``gc`` in a loader worker
started after the GPU tier).

``fork_safe()`` wraps the ``Process.start()`` calls. It first collects the parent's garbage in
the parent, then freezes every object it still tracks (``gc.freeze``: the permanent
generation) across the forks. Each child then only ever collects objects it created itself.
The parent unfreezes afterwards. This is the fork recipe of the ``gc`` module documentation.
"""
import contextlib
import gc


@contextlib.contextmanager
def fork_safe():
    gc.collect()
    gc.freeze()
    try:
        yield
    finally:
        gc.unfreeze()
