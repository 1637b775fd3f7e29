"""mythril_amd — MI355X-native batched path-feasibility engine for Mythril's LASER hot path.

Layers:
  ir      flat register bytecode (mirror of include/pf_bytecode.h)
  lower   bit-vector DAG -> bytecode (register allocation)
  engine  ctypes driver of libpathfeas.so (HIP kernels for gfx950)
  synth   synthetic workloads of BASELINE.json's configs
"""

__version__ = "0.1.0"
