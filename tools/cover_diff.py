"""Which footprints of a covering batch differ from the oracle (status, cell
count, cells, area bits), under each covering knob setting -- a debugging aid
for the general pipeline (GPU).  usage: python tools/cover_diff.py [seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def batch(seed):
    from test_gpu_cover_general import _base_footprints
    rng = np.random.default_rng(seed)
    base = _base_footprints(rng)
    reps = 20000 // len(base) + 1
    polys = []
    for r in range(reps):
        for p in base:
            if r == 0:
                polys.append(p)
                continue
            j = rng.normal(0, 2e-6, size=(len(p), 2))
            polys.append([(float(np.clip(la + dj[0], -90, 90)), float(((ln + dj[1] + 180) % 360) - 180))
                          for (la, ln), dj in zip(p, j)])
    kind = np.zeros(len(polys), np.int32)
    voff = np.zeros(len(polys) + 1, np.int64)
    voff[1:] = np.cumsum([len(p) for p in polys])
    lat = np.array([q[0] for p in polys for q in p], dtype=np.float64)
    lng = np.array([q[1] for p in polys for q in p], dtype=np.float64)
    return kind, voff, lat, lng, np.zeros(len(polys), np.float32)


def main():
    from dss_amd import _lib, geo
    from oracle import oracle as O
    O.build()
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    kind, voff, lat, lng, rad = batch(seed)
    offs, cells, status, area = O.cover_batch(kind, voff, lat, lng, rad)
    area = np.asarray(area, np.float64)
    ctx = _lib.context(0)
    for knobs in ({}, {"cover_slot_order": 0}, {"cover_exact_setup": 1}, {"cover_slot_order": 0, "cover_exact_setup": 1}):
        for k, v in knobs.items():
            ctx.set_tuning(k, v)
        r = geo.cover_batch(kind, voff, lat, lng, rad)
        ctx.set_tuning("cover_slot_order", 1)
        ctx.set_tuning("cover_exact_setup", 0)
        bad = np.nonzero((r.status != status) | (np.diff(r.offs) != np.diff(offs)) |
                         (r.area_km2.view(np.uint64) != area.view(np.uint64)))[0]
        print(knobs, "differing footprints:", len(bad))
        for f in bad[:6]:
            v = slice(voff[f], voff[f + 1])
            print(f"  f={f} nv={voff[f + 1] - voff[f]} status {r.status[f]}/{status[f]} cells "
                  f"{r.offs[f + 1] - r.offs[f]}/{offs[f + 1] - offs[f]} area {r.area_km2[f]!r}/{area[f]!r}")
            print("   lat", lat[v].tolist(), "lng", lng[v].tolist())


if __name__ == "__main__":
    main()
