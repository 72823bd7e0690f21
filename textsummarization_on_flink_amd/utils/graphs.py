"""hipGraph capture hygiene.

``torch.cuda.graph`` no longer runs ``gc.collect()`` before a capture (torch 2.10 only does with
``torch.compiler.config.force_cudagraph_gc``).  An engine dropped earlier in the process that sits
in a reference cycle (a trainer and its phase objects, closures over ``self``) is then freed
whenever the cyclic collector happens to run -- possibly in the middle of another capture, where
the destructors of its CUDAGraphs / events issue HIP calls that a capturing stream does not permit,
and the process aborts ("Fatal Python error: Aborted ... Garbage-collecting" inside a captured
kernel call, seen in a GPU test run in round 4).  ``capture_guard`` collects first and keeps the
collector paused for the whole capture sequence.
"""
from __future__ import annotations

import contextlib
import gc


@contextlib.contextmanager
def capture_guard():
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
