"""testudo_amd -- MI355X-native sqrt-PST polynomial commitments on BLS12-377.

The compute path is libtpst.so (HIP kernels for gfx950 behind the C-ABI of
include/tpst.h); this package is the host-side binding and the mirror of the
reference's sqrt-PST surface (``Polynomial.from_evaluations / commit / open /
verify``, sqrt_pst.rs:14-265).
"""
from .engine import Context, Gens, TpstError  # noqa: F401
