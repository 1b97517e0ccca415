"""Count MFMAs whose destination quad partially overlaps their srcC quad in an
assembly listing (hipcc --cuda-device-only -S).  Round 6 found such MFMAs in a
kernel whose accumulators came out wrong at random (profiles/r6_light_pair.txt).

    python3 scripts/mfma_overlap.py listing.s"""
import re
import sys

tot = bad = 0
for line in open(sys.argv[1]):
    m = re.search(r"v_mfma\w*\s+[va]\[(\d+):(\d+)\],\s*[va]\[?\d+[:\d]*\]?,\s*[va]\[?\d+[:\d]*\]?,"
                  r"\s*[va]\[(\d+):(\d+)\]", line)
    if m:
        tot += 1
        d0, d1, c0, c1 = map(int, m.groups())
        if (d0, d1) != (c0, c1) and not (d1 < c0 or c1 < d0):
            bad += 1
print(f"{sys.argv[1]}: {tot} MFMAs, {bad} with dst partially overlapping srcC")
