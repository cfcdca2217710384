"""Host BAM ingest alone (no GPU): the product's streaming decode of a synthetic
coordinate-sorted BAM into batch slots, as `CellProcessor.run_stream` drives it
(64-byte records, BAM order, no placement), timed over a few passes.

    python scripts/decode_bench.py [--reads N] [--cells C] [--threads T] [--passes P]

MGP_HOST_PROFILE=1 prints the decoder's stage times per pass.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--cells", type=int, default=1_000)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4_000_000)
    ap.add_argument("--out", default="/tmp/mgp_decode_bench")
    args = ap.parse_args()

    from mgatk2_amd.bam import BamFile, StreamSlot, host_threads, write_bam
    from mgatk2_amd.synth import barcode_names, synth_reads

    out = Path(args.out)
    out.mkdir(parents=True, exist_ok=True)
    seed = 20251015 + 3
    whitelist = barcode_names(args.cells, seed)
    bam = out / f"d_{args.reads}_{args.cells}.bam"
    if not bam.exists():
        t = time.time()
        soa = synth_reads(seed, args.reads, args.cells, pack=False)
        write_bam(bam, soa, whitelist, level=6)
        del soa
        print(f"[decode] BAM {bam.stat().st_size / 1e9:.2f} GB written in {time.time() - t:.1f}s", file=sys.stderr)
    nt = args.threads or host_threads()
    slot = StreamSlot(args.batch, args.batch * 64 + (64 << 20))
    times = []
    for _ in range(args.passes):
        t = time.time()
        n = 0
        with BamFile(bam, n_threads=nt) as bf, bf.stream("chrM", whitelist, paired=False) as st:
            while True:
                got = st.next_into(slot)
                if not got:
                    break
                n += slot.n
        times.append(time.time() - t)
    print(json.dumps({"reads": n, "threads": nt, "bam_bytes": bam.stat().st_size, "seconds": [round(x, 3) for x in times],
                      "ns_per_read_thread": round(min(times) * nt / max(n, 1) * 1e9, 1)}))


if __name__ == "__main__":
    main()
