"""pntf — MI355X-native hot path of P-NTFields (τ / ∇τ fields, path velocity, planner).

Host runtime for libpntf.so (HIP, gfx950).  `pntf.ops` holds the torch-facing entry
points, `pntf.net` the pieces shared by the drop-in `models` modules, `pntf.synth` the
seeded synthetic inputs, `pntf.dist` the multi-GPU sharding.
"""
__version__ = "0.1.0"
