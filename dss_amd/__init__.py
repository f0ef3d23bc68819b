"""dss_amd: MI355X-native engine for the InterUSS DSS spatial-discovery and
4D-conflict hot path (level-13 S2 covering + overlap search).

Product entry points: dss_amd.geo (covering API), dss_amd.store (search API),
dss_amd.device (HBM-resident batch API).  All compute runs in
libdss_amd.so (gfx950 HIP kernels); there is no CPU fallback.
"""
__all__ = ["geo", "store", "workload"]
