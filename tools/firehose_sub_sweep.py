#!/usr/bin/env python3
"""One GPU's share of the configs[2] firehose at 8 GPUs (2,097,152 signatures) verified as
resident sub-shards of different sizes (bench.firehose_pass): per-GPU throughput by sub-shard
size, the data behind bench.firehose_subshard."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import narwhal_amd  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 2097152
    eng = narwhal_amd.Engine(device=0)
    for sub in (2097152, 1048576, 524288, 262144):
        if sub > m:
            continue
        os.environ["NWV_FIREHOSE_SUBSHARD"] = str(sub)
        dt, _, kt, nsub = bench.firehose_pass(eng, 0, m, 6, warm=2)
        print(json.dumps({"sigs": m, "subshard": sub, "subshards": nsub, "passes": 6,
                          "ms_per_pass": dt / 6 * 1e3, "sigs_per_s": m * 6 / dt,
                          "kernel_ms_one_subshard": kt}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
