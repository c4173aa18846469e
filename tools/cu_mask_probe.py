#!/usr/bin/env python3
"""Map hipExtStreamCreateWithCUMask bits to physical CUs (XCC / SE / CU) on the GPU.

Runs the placement probe on a plain stream and on streams whose CU mask clears
(a) the top 8 bits, (b) bit 31 of every 32-bit word, (c) bits 0..7, and
reports, per XCC, how many distinct CUs each stream reached.
"""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import heat3d_amd

    ext = heat3d_amd.native()
    full = [0xFFFFFFFF] * 8
    cases = {"plain": [], "all_bits": full,
             "clear_top8": full[:7] + [0x00FFFFFF],
             "clear_bit31_each_word": [0x7FFFFFFF] * 8,
             "clear_low8": [0xFFFFFF00] + full[1:],
             "clear_word0": [0] + full[1:]}
    out = {}
    for name, m in cases.items():
        ids = ext.cu_mask_probe(0, m, 8192)
        per = collections.Counter(i >> 8 for i in ids)
        out[name] = {"cus": len(ids), "per_xcc": dict(sorted(per.items()))}
        print(name, json.dumps(out[name]), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
