"""Reader for the Tecplot ASCII files written by heat3d (and the reference's
output/out.dat, heat3D.cu:1125-1179)."""
from __future__ import annotations

import re
from typing import Dict, List

import numpy as np

_ZONE = re.compile(r'ZONE T = "(\d+)", I=(\d+), J=(\d+), K=(\d+), F=POINT')


def read_tecplot(path: str) -> Dict:
    with open(path, "r") as f:
        lines = f.read().splitlines()
    if not lines or not lines[0].startswith("TITLE="):
        raise ValueError("not a Tecplot file")
    variables = re.findall(r'"(\w+)"', lines[1])
    zones: List[Dict] = []
    i = 2
    while i < len(lines):
        m = _ZONE.match(lines[i])
        if not m:
            raise ValueError(f"line {i + 1}: expected ZONE header, got {lines[i]!r}")
        title, I, J, K = (int(v) for v in m.groups())
        cnt = I * J * K
        rows = lines[i + 1: i + 1 + cnt]
        data = np.array([[float(x) for x in r.split()] for r in rows], dtype=np.float64)
        zones.append({"title": title, "shape": (I, J, K), "data": data})
        i += 1 + cnt
    return {"variables": variables, "zones": zones}
