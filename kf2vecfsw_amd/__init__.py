"""kf2vecfsw_amd -- MI355X-native replacement of kf2vec's k-mer frequency-vector
builder (`get_frequencies`, reference kf2vec/main.py:250-373).

Layout:
  csrc/kf_count.hip   HIP kernels (gfx950) + device half of the C-ABI
  csrc/kf_host.cpp    host half of the C-ABI (tables, record index, .kf writer)
  _native.py          ctypes binding of libkf2vec_gpu.so (no CPU fallback)
  counter.py          batch packing + KmerCounter (device counting)
  main.py             `get_frequencies` CLI mirror
"""
__all__ = ["__version__"]
__version__ = "0.1.0"
