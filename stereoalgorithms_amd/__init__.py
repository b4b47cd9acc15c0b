"""stereoalgorithms_amd — MI355X-native stereo depth engine (RAFT-Stereo, CREStereo, HITNet,
Fast-ACVNet+), with the capabilities of LiuWQ0809/StereoAlgorithms re-designed for CDNA4.

Layers:
  * ``csrc/``                native C++/HIP: kernels, engine runtime, models, C ABI, geometry
  * ``stereoalgorithms_amd._native``  ctypes bindings to the in-tree libraries
  * ``ops``                  torch-facing kernel wrappers (tests / tooling)
  * ``models``               PyTorch oracles + native engine handle
  * ``parallel``             data-parallel frame sharding over torch.distributed (RCCL)
  * ``utils``                calibration YAML, geometry, image / point-cloud I/O, weights
"""
__version__ = "0.1.0"
