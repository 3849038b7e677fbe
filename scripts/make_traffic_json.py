#!/usr/bin/env python3
"""HBM traffic per launch of the route kernel from rocprofv3 PMC passes -> profiles/route_kernel_pmc.json.

Corrections (profiles/r01_pmc_calibration.txt, MI355X_MICROARCH.md §HBM): FETCH_SIZE tallies every read request at
64 B; streaming 128-B requests are therefore under-counted by 2x, so the header stream (32 B x messages, read once,
coalesced) is added back once; random 32-B directory probes are one 64-B request each and are counted as tallied.
WRITE_SIZE is exact for the kernel's 4-B/lane coalesced stores.  Bytes served by the Infinity Cache are included
(the counters sit on the L2's memory side), so this is an upper bound on DRAM bytes.

Usage: python scripts/make_traffic_json.py gpurun_out/prof MSGS_PER_LAUNCH [out.json] [CONFIG]
(run here, on the pulled PMC passes: the record carries the config and the git build it was measured at, which bench.py
checks before it quotes the traffic)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    prof, msgs = sys.argv[1], int(float(sys.argv[2]))
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "route_kernel_pmc.json")
    config = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    try:
        build = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                               check=True).stdout.strip()
    except Exception:
        build = None
    tmp = os.path.join(prof, "pmc_summary.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), prof, "--json", tmp], check=True,
                   stdout=subprocess.DEVNULL)
    s = json.load(open(tmp))
    k = next(n for n in s if n.startswith("orl::k_route"))
    c = s[k]
    header = 32 * msgs
    fetch = c["FETCH_SIZE"] * 1024 + header / 2
    write = c["WRITE_SIZE"] * 1024
    rec = {"kernel": k, "config": config, "build": build, "msgs_per_launch": float(msgs), "hbm_bytes_per_launch": fetch + write,
           "read_bytes": fetch, "write_bytes": write, "algorithmic_bytes": 72.0 * msgs,
           "tcc_ea0_rdreq": c.get("TCC_EA0_RDREQ_sum"), "tcc_hit": c.get("TCC_HIT_sum"), "tcc_miss": c.get("TCC_MISS_sum"),
           "method": "FETCH_SIZE*1024 + 16 B/msg streaming correction + WRITE_SIZE*1024 (scripts/make_traffic_json.py)"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
