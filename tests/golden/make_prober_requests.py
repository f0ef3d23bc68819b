"""Writes tests/golden/prober_requests.json: the request bodies of the
reference's prober fixtures monitoring/prober/scd/resources/op_request_{1,2,3}.json
(data only), so the GPU tests can replay them on a box without /root/reference."""
import json
import os

REF = "/root/reference/monitoring/prober/scd/resources"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "prober_requests.json")

if __name__ == "__main__":
    d = {}
    for k in (1, 2, 3):
        with open(os.path.join(REF, f"op_request_{k}.json")) as f:
            d[f"op_request_{k}"] = json.load(f)
    with open(OUT, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print("wrote", OUT)
