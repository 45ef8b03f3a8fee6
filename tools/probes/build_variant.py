"""Build an experiment variant of libsurprise_amd.so with extra -D switches (timing A/B only):
    python tools/probes/build_variant.py NAME -DSWITCH[=V] ...  -> tests/variants/libsurprise_amd_NAME.so
Load it with SURPRISE_AMD_LIB=<path> (the loader then skips the source-hash check)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from surprise_amd import build  # noqa: E402

name, extra = sys.argv[1], tuple(sys.argv[2:])
out = os.path.join(ROOT, "tests", "variants", "libsurprise_amd_%s.so" % name)
os.makedirs(os.path.dirname(out), exist_ok=True)
print(build.build(out=out, extra=extra))
