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
import os as _os

# ROCm's graph "packet capture" fast path (AQL packets + kernel arguments pre-baked at
# instantiation) corrupted replays of our captured frames when other HIP work (torch kernels
# loading new code objects) ran between replays: garbage disparities and, downstream, illegal
# memory accesses (reproduced by tests/test_raft_engine_gpu.py::test_engine_cloud_and_rectify_roundtrip;
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 makes it pass).  The runtime reads the flag once at HIP
# initialisation, so it is set here, before torch initialises the device, and by a load-time
# constructor in libstereo_amd.so for the C/C++ entry points.
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

__version__ = "0.1.0"
