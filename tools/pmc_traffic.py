"""Per-launch HBM traffic and executed fp64 work of the rollout kernel from rocprofv3 PMC passes
(tools/gpu_pmc.sh), written to a JSON that bench.py reports as roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md (HBM section) gfx950's
FETCH_SIZE tallies 128-B requests at 64 B, so it is doubled here; the rollout kernel's reads are
8-B-per-lane eps loads (a width the guide leaves uncalibrated) - the doubled figure agrees with
the 25.2 MB eps tensor, which is the check that the correction applies.

usage: pmc_traffic.py <pmc dir> <out.json> [kernel name part]   (default: the rollout launch, "[main]")
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import summarize  # noqa: E402


def main(d, out, prefix=None):
    fetch = summarize(d + "/fetch_counter_collection.csv")
    write = summarize(d + "/write_counter_collection.csv")
    flops = summarize(d + "/flops_counter_collection.csv")
    key = [k for k in fetch if ((prefix in k) if prefix else k.endswith("[main]"))][0]
    kib = 1024.0
    f = fetch[key]["FETCH_SIZE"] * kib * 2.0
    w = write[key]["WRITE_SIZE"] * kib
    res = {
        "kernel": key,
        "fetch_bytes": f,
        "write_bytes": w,
        "traffic_bytes": f + w,
        "fp64_wave_flops": flops[key]["SQ_INSTS_VALU_FLOPS_FP64"],
        "fp64_executed_flops": flops[key]["SQ_INSTS_VALU_FLOPS_FP64"] * 64.0,
        "note": "per launch; FETCH_SIZE doubled (gfx950); executed flops = wave-instruction flops x 64 lanes",
        "source": d,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
