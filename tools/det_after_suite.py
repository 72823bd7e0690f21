"""Run the GPU test tier, then (same process, same allocator state) compare two deterministic-mode
graph trainers buffer by buffer with tools/det_diff.py's logic -- for a divergence that only
shows after the rest of the suite has run.

  python tools/det_after_suite.py [pytest args...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pytest  # noqa: E402


def main():
    args = sys.argv[1:] or ["tests", "-m", "gpu", "-q", "--timeout", "300", "--timeout-method", "thread",
                            "-k", "not deterministic"]
    rc = pytest.main(args)
    print("suite rc", rc, flush=True)
    os.environ["TSAMD_DETERMINISTIC"] = "1"
    sys.argv = [sys.argv[0], "--iters", "5", "--graph"]
    import runpy
    runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "det_diff.py"), run_name="__main__")


if __name__ == "__main__":
    main()
