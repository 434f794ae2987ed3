"""The rejected k <= 8 kernel variants of rounds 1-2 (tools/zoo/kf_count_zoo.hip,
KF_COUNT_VARIANT) as their own library, tools/zoo/libkf2vec_zoo.so (built by
`python -m kf2vecfsw_amd.build --zoo`).  Not part of the product; run on a GPU
box with `pytest tools/zoo -m gpu`."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["KF2VEC_GPU_LIB"] = os.path.join(ROOT, "tools", "zoo", "libkf2vec_zoo.so")
from conftest import *  # noqa: E402,F401,F403  (fixtures: native, oracle, toy)
