"""MI355X-native batched replay engine for the Fluid Framework merge-tree (SharedString / SharedMatrix).

The hot path -- applying sequenced merge-tree ops (`Client.applyMsg`) and producing the SnapshotV1
summary -- runs as hand-written HIP kernels on gfx950 behind the C ABI in include/mtb.h.
"""
from .client import Client, MatrixBatch, MergeTreeBatch, MergeTreeError, SharedMatrix, UsageError  # noqa: F401
