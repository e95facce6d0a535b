"""GPU box: one tools/soak.py case with the parity assertion's message (which field differs)."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
args = sys.argv[1:]
sys.argv = [sys.argv[0], "0"]
import soak  # noqa: E402

try:
    getattr(soak, "fam_" + args[0])(int(args[1]))
    print(args, "ok")
except Exception as e:
    print(args, "".join(traceback.format_exception_only(type(e), e))[:3000])
