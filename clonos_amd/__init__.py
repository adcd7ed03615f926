"""clonos_amd -- MI355X-native causal-log engine for Clonos (decode, delta-slice, truncate,
replay-prep on gfx950).  The compute path is libclonos_engine.so (HIP); this package is
the host-side mirror of the reference Java interfaces."""
from . import determinants
from ._lib import ClonosError
from .engine import CausalLogID, DecodedBatch, Engine, ThreadCausalLog

__all__ = ["Engine", "ThreadCausalLog", "CausalLogID", "DecodedBatch", "ClonosError", "determinants"]
