"""Seeded synthetic workloads for the BASELINE.json configs.

numpy default_rng(seed), seed = 20201015 + i with i the index in
BASELINE.json `configs`.  All outputs are flat numpy arrays in the layout the
C ABI takes (kind, voff, lat, lng, radius_m for footprints; SoA attributes).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

KIND_POLYGON = 0
KIND_CIRCLE = 1
T0_US = 1_600_000_000_000_000  # "T" of the generator: an arbitrary UTC instant (2020-09-13)
HOUR_US = 3_600_000_000
MIN_US = 60_000_000
R_EARTH = 6371010.0

METRO = (37.2, 37.9, -122.55, -121.75)       # SF Bay (configs 0, 1)
CALIFORNIA = (32.5, 42.0, -124.4, -114.1)    # config 2
NYC = (40.49, 40.92, -74.26, -73.70)         # config 3
CONUS = (25.0, 49.0, -124.5, -67.0)          # config 4
CA_HOTSPOTS = [(34.05, -118.25), (37.77, -122.42), (32.72, -117.16), (38.58, -121.49)]


@dataclass
class Footprints:
    kind: np.ndarray      # int32 [n]
    voff: np.ndarray      # int64 [n+1]
    lat: np.ndarray       # float64 [voff[n]]
    lng: np.ndarray       # float64
    radius_m: np.ndarray  # float32 [n]

    @property
    def n(self) -> int:
        return len(self.kind)

    def slice(self, a: int, b: int) -> "Footprints":
        """Footprints [a, b) (vertex offsets rebased to 0)."""
        v0, v1 = int(self.voff[a]), int(self.voff[b])
        return Footprints(self.kind[a:b], self.voff[a:b + 1] - v0, self.lat[v0:v1], self.lng[v0:v1],
                          self.radius_m[a:b])

    def subset(self, idx: np.ndarray) -> "Footprints":
        idx = np.asarray(idx)
        counts = self.voff[idx + 1] - self.voff[idx]
        voff = np.zeros(len(idx) + 1, dtype=np.int64)
        np.cumsum(counts, out=voff[1:])
        take = np.concatenate([np.arange(self.voff[i], self.voff[i + 1]) for i in idx]) if len(idx) else np.zeros(0, np.int64)
        return Footprints(self.kind[idx].copy(), voff, self.lat[take].copy(), self.lng[take].copy(),
                          self.radius_m[idx].copy())


def _offset(lat0, lng0, dx, dy):
    """Local tangent-plane offset (metres east dx, north dy) -> degrees."""
    dlat = np.degrees(dy / R_EARTH)
    dlng = np.degrees(dx / (R_EARTH * np.cos(np.radians(lat0))))
    return lat0 + dlat, lng0 + dlng


def _centres(rng, n, region, hotspots=None, hot_frac=0.0, sigma_m=15000.0):
    la0, la1, ln0, ln1 = region
    lat = rng.uniform(la0, la1, n)
    lng = rng.uniform(ln0, ln1, n)
    if hotspots and hot_frac > 0:
        hot = rng.random(n) < hot_frac
        k = rng.integers(0, len(hotspots), n)
        hs = np.asarray(hotspots)
        dx = rng.normal(0, sigma_m, n)
        dy = rng.normal(0, sigma_m, n)
        hl, hg = _offset(hs[k, 0], hs[k, 1], dx, dy)
        lat = np.where(hot, np.clip(hl, la0, la1), lat)
        lng = np.where(hot, np.clip(hg, ln0, ln1), lng)
    return lat, lng


def metro_footprints(rng, n, region=METRO, circle_frac=0.3, hotspots=None, hot_frac=0.0, sigma_m=15000.0,
                     rmin=100.0, rmax=3000.0) -> Footprints:
    """Polygons (V ~ U{3..12}, radius ~ logU[rmin, rmax], radial jitter
    U[0.6, 1.0], 50% clockwise, 25% closed rings) and circles (radius f32 ~
    U[50, 2000] m), polygon:circle = (1-circle_frac):circle_frac."""
    clat, clng = _centres(rng, n, region, hotspots, hot_frac, sigma_m)
    is_circle = rng.random(n) < circle_frac
    nv = rng.integers(3, 13, n)
    closed = (rng.random(n) < 0.25) & ~is_circle
    cw = rng.random(n) < 0.5
    radius = np.exp(rng.uniform(np.log(rmin), np.log(rmax), n))
    counts = np.where(is_circle, 1, nv + closed.astype(np.int64))
    voff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=voff[1:])
    tot = int(voff[-1])
    lat = np.empty(tot)
    lng = np.empty(tot)
    # vectorised polygon construction: angles theta0 + 2*pi*k/nv with a
    # +-0.2-spacing jitter, so consecutive gaps stay < pi and the polygon is
    # star-shaped about its centre, hence simple (the generator contract's
    # "sorted U[0,2pi) angles" can produce self-intersecting, i.e. invalid,
    # S2 loops whose parity interior is most of the sphere).
    maxv = 13
    col = np.arange(maxv)[None, :]
    valid = col < nv[:, None]
    spacing = 2 * np.pi / nv[:, None]
    ang = rng.uniform(0, 2 * np.pi, (n, 1)) + spacing * (col + rng.uniform(-0.2, 0.2, (n, maxv)))
    jit = rng.uniform(0.6, 1.0, (n, maxv))
    # clockwise: reverse vertex order among the first nv
    rev_idx = np.where(valid, nv[:, None] - 1 - col, col)
    ang = np.where(cw[:, None], np.take_along_axis(ang, rev_idx, axis=1), ang)
    jit = np.where(cw[:, None], np.take_along_axis(jit, rev_idx, axis=1), jit)
    r = radius[:, None] * jit
    plat, plng = _offset(clat[:, None], clng[:, None], r * np.cos(ang), r * np.sin(ang))
    poly = ~is_circle
    rows = np.repeat(np.arange(n)[poly], nv[poly])
    cols = np.concatenate([np.arange(v) for v in nv[poly]]) if poly.any() else np.zeros(0, np.int64)
    dst = voff[rows] + cols
    lat[dst] = plat[rows, cols]
    lng[dst] = plng[rows, cols]
    cidx = np.nonzero(closed)[0]
    lat[voff[cidx] + nv[cidx]] = lat[voff[cidx]]
    lng[voff[cidx] + nv[cidx]] = lng[voff[cidx]]
    ci = np.nonzero(is_circle)[0]
    lat[voff[ci]] = clat[ci]
    lng[voff[ci]] = clng[ci]
    radius_m = np.where(is_circle, rng.uniform(50.0, 2000.0, n), 0.0).astype(np.float32)
    kind = np.where(is_circle, KIND_CIRCLE, KIND_POLYGON).astype(np.int32)
    return Footprints(kind, voff, lat, lng, radius_m)


def _quads(rng, n, clat, clng, a, b, rot, cw):
    """4-gons centred at (clat, clng): half-extents a (along rot) and b
    (across), CCW unless cw.  Returns Footprints."""
    corners = np.array([[-1, -1], [1, -1], [1, 1], [-1, 1]], dtype=np.float64)
    order = np.where(cw[:, None], np.array([3, 2, 1, 0])[None, :], np.array([0, 1, 2, 3])[None, :])
    cx = corners[order, 0] * a[:, None]
    cy = corners[order, 1] * b[:, None]
    c, s = np.cos(rot)[:, None], np.sin(rot)[:, None]
    dx = cx * c - cy * s
    dy = cx * s + cy * c
    plat, plng = _offset(clat[:, None], clng[:, None], dx, dy)
    voff = np.arange(n + 1, dtype=np.int64) * 4
    return Footprints(np.full(n, KIND_POLYGON, np.int32), voff, plat.reshape(-1).copy(), plng.reshape(-1).copy(),
                      np.zeros(n, np.float32))


def city_blocks(rng, n, region=NYC) -> Footprints:
    """city-block 4-gons, sides U[80, 250] m, rotated
    U[0, 30] degrees, half of them clockwise (reversal path)."""
    clat, clng = _centres(rng, n, region)
    a = rng.uniform(80, 250, n) / 2
    b = rng.uniform(80, 250, n) / 2
    rot = np.radians(rng.uniform(0, 30, n))
    cw = rng.random(n) < 0.5
    return _quads(rng, n, clat, clng, a, b, rot, cw)


CONUS_HOTSPOTS = [(40.71, -74.01), (34.05, -118.24), (41.88, -87.63), (29.76, -95.37), (33.45, -112.07),
                  (39.95, -75.17), (29.42, -98.49), (32.72, -117.16), (32.78, -96.80), (37.34, -121.89),
                  (30.27, -97.74), (39.74, -104.99), (47.61, -122.33), (42.36, -71.06), (38.91, -77.04),
                  (36.17, -86.78), (45.52, -122.68), (25.76, -80.19), (33.75, -84.39), (44.98, -93.27)]


def corridors(rng, n, region=CONUS, hotspots=CONUS_HOTSPOTS, hot_frac=0.8, sigma_m=20000.0) -> Footprints:
    """long thin 4-gon corridors, length logU[5, 100]
    km, width U[30, 300] m, orientation U[0, pi), 80% around 20 metro
    hotspots (sigma 20 km), half of them clockwise."""
    clat, clng = _centres(rng, n, region, hotspots, hot_frac, sigma_m)
    length = np.exp(rng.uniform(np.log(5000.0), np.log(100000.0), n))
    width = rng.uniform(30, 300, n)
    rot = rng.uniform(0, np.pi, n)
    cw = rng.random(n) < 0.5
    return _quads(rng, n, clat, clng, length / 2, width / 2, rot, cw)


@dataclass
class Attrs:
    alt_lo: np.ndarray  # float32
    alt_hi: np.ndarray
    t0: np.ndarray      # int64 us (NULL start -> INT64_MIN)
    t1: np.ndarray      # int64 us (NULL end  -> INT64_MAX for queries)


def intent_attrs(rng, n) -> Attrs:
    lo = rng.uniform(0, 400, n).astype(np.float32)
    hi = (lo + rng.uniform(10, 200, n)).astype(np.float32)
    t0 = T0_US + rng.integers(0, 24 * HOUR_US, n)
    t1 = t0 + rng.integers(5 * MIN_US, 2 * HOUR_US + 1, n)
    return Attrs(lo, hi, t0.astype(np.int64), t1.astype(np.int64))


def query_attrs(rng, n) -> Attrs:
    lo = rng.uniform(0, 400, n).astype(np.float32)
    hi = (lo + rng.uniform(10, 200, n)).astype(np.float32)
    miss = rng.random(n) < 0.05           # Q8: missing SCD altitude -> 0.0
    lo = np.where(miss, np.float32(0), lo).astype(np.float32)
    hi = np.where(miss, np.float32(0), hi).astype(np.float32)
    t0 = T0_US + rng.integers(0, 24 * HOUR_US, n)
    t1 = t0 + rng.integers(1 * MIN_US, 30 * MIN_US + 1, n)
    nulls = rng.random(n) < 0.05
    which = rng.random(n) < 0.5
    t0 = np.where(nulls & which, np.iinfo(np.int64).min, t0)
    t1 = np.where(nulls & ~which, np.iinfo(np.int64).max, t1)
    return Attrs(lo, hi, t0.astype(np.int64), t1.astype(np.int64))


def rid_attrs(rng, n, query: bool) -> Attrs:
    """ISAs t0 = T + U[0, 1 h), 30 s long;
    queries earliest = T + U[0, 1 h), latest = earliest + 30 s.  RID search
    has no altitude predicate (identification_service_area.go:170-180), so
    altitudes are the NULL sentinels."""
    t0 = T0_US + rng.integers(0, HOUR_US, n)
    t1 = t0 + 30_000_000
    inf = np.full(n, np.inf, np.float32)
    return Attrs(-inf, inf, t0.astype(np.int64), t1.astype(np.int64))


# BASELINE.json configs: (queries, entities, kind) at scale 1
CONFIG_SIZES = {0: (10_000, 100_000), 1: (1_000_000, 1_000_000), 2: (1_000_000, 10_000_000),
                3: (1_000_000, 5_000_000), 4: (1_000_000, 50_000_000)}
# (workload descriptions only: the GPU count of a line is its n_gpus)
CONFIG_NAMES = {0: "Go CPU ref workload: SF-Bay metro, circles+polygons",
                1: "metro: SF-Bay, circles+polygons",
                2: "north-star airspace: California, 70% around 4 hotspots",
                3: "RID ISAs: NYC city blocks, 30 s windows",
                4: "continent stress: CONUS corridors, 80% around 20 hotspots"}


def config(i: int, scale: float = 1.0):
    """Return (rng, queries, q_attrs, intents, i_attrs, now_us) for BASELINE config i.

    `scale` shrinks the counts (tests); the shapes and distributions stay.
    Config 3 is RID (search_isas semantics: no altitude, 30 s windows)."""
    rng = np.random.default_rng(20201015 + i)
    if i not in CONFIG_SIZES:
        raise ValueError(f"config {i} not generated here")
    nq, ni = CONFIG_SIZES[i]
    nq = max(1, int(nq * scale))
    ni = max(1, int(ni * scale))
    if i in (0, 1, 2):
        kw = dict(hotspots=CA_HOTSPOTS, hot_frac=0.7, sigma_m=15000.0) if i == 2 else {}
        region = CALIFORNIA if i == 2 else METRO
        intents = metro_footprints(rng, ni, region, **kw)
        ia = intent_attrs(rng, ni)
        queries = metro_footprints(rng, nq, region, **kw)
        qa = query_attrs(rng, nq)
    elif i == 3:
        intents = city_blocks(rng, ni)
        ia = rid_attrs(rng, ni, False)
        queries = city_blocks(rng, nq)
        qa = rid_attrs(rng, nq, True)
    else:
        intents = corridors(rng, ni)
        ia = intent_attrs(rng, ni)
        queries = corridors(rng, nq)
        qa = query_attrs(rng, nq)
    return rng, queries, qa, intents, ia, T0_US


def _footprints_for(i: int, rng, n: int) -> Footprints:
    if i in (0, 1):
        return metro_footprints(rng, n, METRO)
    if i == 2:
        return metro_footprints(rng, n, CALIFORNIA, hotspots=CA_HOTSPOTS, hot_frac=0.7, sigma_m=15000.0)
    if i == 3:
        return city_blocks(rng, n)
    return corridors(rng, n)


def config_split(i: int, rank: int = 0, scale: float = 1.0, queries_scale: float = 1.0):
    """bench.py's form of config i: the airspace (entities + attributes) from
    the config's seed, identical on every rank, and a rank-private query batch
    (seed 20201015 + i + 1000 * (rank + 1)) of the config's query shape.
    Returns (queries, q_attrs, entities, e_attrs, now_us, rid)."""
    if i not in CONFIG_SIZES:
        raise ValueError(f"config {i} not generated here")
    nq, ni = CONFIG_SIZES[i]
    nq = max(1, int(nq * scale * queries_scale))
    ni = max(1, int(ni * scale))
    rid = i == 3
    rng_i = np.random.default_rng(20201015 + i)
    ents = _footprints_for(i, rng_i, ni)
    ea = rid_attrs(rng_i, ni, False) if rid else intent_attrs(rng_i, ni)
    rng_q = np.random.default_rng(20201015 + i + 1000 * (rank + 1))
    qs = _footprints_for(i, rng_q, nq)
    qa = rid_attrs(rng_q, nq, True) if rid else query_attrs(rng_q, nq)
    return qs, qa, ents, ea, T0_US, rid


def query_bounds(qa: Attrs, now_us: int):
    """Query (tlo, thi) as the search kernels take them: SCD
    `COALESCE(ends_at >= start) AND ends_at >= now` (operations.go:398-402)
    and the RID app-layer clamp earliest = max(now, earliest) (isa.go:38-45)
    both fold into tlo = max(t0, now)."""
    return np.maximum(qa.t0, now_us), qa.t1
