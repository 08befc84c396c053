"""pinot_amd: MI355X-native Pinot segment query hot path (filter -> projection -> aggregation / group-by).

Product path: pinot_amd.gpu (libpinot_gpu.so, hand-written HIP for gfx950) behind the C ABI in
include/pinot_gpu.h.  Host-side mirror of the reference's query interface: pinot_amd.query
(QueryContext), pinot_amd.plan (predicate lowering / plan maker / reduce), pinot_amd.segment
(on-disk segment formats).
"""
__all__ = ["segment", "query", "plan", "abi", "gpu"]
