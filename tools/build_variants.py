"""Build experiment variants of the library into build_exp/ (name=-Dflags ...), e.g.
python tools/build_variants.py nolog=-DMF_EXP_NO_LOG_STORE nt=-DMF_LOG_AUX=2"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from surprise_amd import build  # noqa: E402

os.makedirs(os.path.join(ROOT, "build_exp"), exist_ok=True)
for arg in sys.argv[1:]:
    name, _, flags = arg.partition("=")
    out = os.path.join(ROOT, "build_exp", f"lib_{name}.so")
    print(build.build(force=True, out=out, extra=tuple(flags.split())), flush=True)
