"""A/B helper: run bench.py's main() with the sdreamer package taken from another directory (e.g. a copy of the
previous commit's Python under _ab/base), against the same libsdhip.so (SDHIP_LIB). Usage:
python tools/ab_bench.py <package_root> [bench args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pkg = os.path.abspath(sys.argv[1])
os.environ.setdefault("SDHIP_LIB", os.path.join(ROOT, "safe-dreamer_amd", "sdreamer", "_lib", "libsdhip.so"))
os.environ.setdefault("SDHIP_HEADER", os.path.join(ROOT, "include", "sdhip.h"))
sys.argv = [sys.argv[0]] + sys.argv[2:]
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (inserts the in-tree package path)

sys.path.insert(0, pkg)
bench.main()
