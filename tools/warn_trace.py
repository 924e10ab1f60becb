"""Run bench.py's main() with every Python warning printed with the stack that raised it (the
AccumulateGrad stream-mismatch warning names no tensor; its stack names the call that triggers it)."""
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def show(message, category, filename, lineno, file=None, line=None):
    print(f"[warn-trace] {category.__name__}: {message}", file=sys.stderr)
    traceback.print_stack(limit=25, file=sys.stderr)


warnings.showwarning = show
warnings.simplefilter("always")
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
