#!/usr/bin/env python3
"""bench.py of another checkout of this repository (e.g. a `git worktree` of the previous commit with its own
in-tree build), for interleaved A/B runs of kernel changes that have no runtime switch:

    AB_SCRIPT=tools/ab_tree.py tools/ab_bench.sh 3 "DTG_AB_TREE=.ab_old" "DTG_AB_TREE=." -- --model bert

The tree's bench.py puts its own directory first on sys.path, so `import dtg` loads that tree's package and .so."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.abspath(os.path.join(ROOT, os.environ.get("DTG_AB_TREE", ".")))
sys.path.insert(0, tree)
sys.argv = [os.path.join(tree, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
