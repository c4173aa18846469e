"""Where the CU mask of the solver's compute stream puts work (VERDICT r2 weak
#8): `reserve_cus(n)` clears the top n bits of the mask
(csrc/runtime/hip_backend.cpp); the docs claim that with n = 8 this keeps one
CU per XCD free for RCCL's channel kernels and the check kernel.  The probe
kernel records (XCC_ID, HW_ID.CU) of every workgroup it runs
(kernels_hip.hip cu_probe_kernel)."""
import collections

import pytest

pytestmark = pytest.mark.gpu


def _per_xcc(ext, mask):
    ids = ext.cu_mask_probe(0, mask, 8192)
    return len(ids), collections.Counter(i >> 8 for i in ids)


def test_cu_mask_bits_round_robin_over_xcds(h3d, gpu):
    ext = h3d.native()
    full = [0xFFFFFFFF] * 8
    n, per = _per_xcc(ext, full)
    assert n == 256 and sorted(per.values()) == [32] * 8, per
    # the solver's reservation: top 8 bits -> one CU on every XCD
    n, per = _per_xcc(ext, full[:7] + [0x00FFFFFF])
    assert n == 248 and sorted(per.values()) == [31] * 8, per
    # bit i lives on XCD i mod 8: bits 31, 63, ..., 255 are all XCD 7
    n, per = _per_xcc(ext, [0x7FFFFFFF] * 8)
    assert n == 248 and per[7] == 24 and all(per[x] == 32 for x in range(7)), per
