"""The evidence keys of bench.py (no GPU needed): per-kernel ISA hashes of the built library
cover both translation units (fast kernels, exact-mode kernels), ignore where a kernel sits in
the code object, and the committed profiles of the headline kernel (profiles/r04) match the library
this tree builds (so the bench line quotes them)."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hashes():
    from rl_rocket_amd import build as B

    if not os.path.exists(B.OUT):
        pytest.skip("librocket_hip.so not built")
    return B.kernel_isa_hashes(B.OUT)


def test_every_translation_unit_hashed(hashes):
    names = list(hashes)
    assert any("step_kernel<6, 0, false, true, 4, false>" in k for k in names)  # main
    assert any("step_exact_kernel<6, true, false>" in k for k in names)  # exact
    assert any("step_exact_kernel<6, false, false>" in k for k in names)
    assert any("rollout_step_kernel<6, 0, 0, false" in k for k in names)  # main
    assert any("rollout_step_kernel<6, 0, 0, true" in k for k in names)  # collect
    assert all(len(v) == 16 for v in hashes.values())


def test_descriptor_offset_is_ignored():
    """Two kernels' descriptors differ in kernel_code_entry_byte_offset by where the code sits;
    the hash zeroes that field (bytes 16..23 of the 64-byte descriptor)."""
    import hashlib

    code = b"\x01\x02\x03\x04" * 8
    kd_a = bytearray(64)
    kd_b = bytearray(64)
    kd_a[16:24] = (1000).to_bytes(8, "little")
    kd_b[16:24] = (5000).to_bytes(8, "little")

    def h(kd):
        kd = bytearray(kd)
        kd[16:24] = bytes(8)
        x = hashlib.sha256(code)
        x.update(bytes(kd))
        return x.hexdigest()

    assert h(kd_a) == h(kd_b)


def test_committed_headline_evidence_matches_this_build(hashes):
    import bench

    traffic, src = bench.stored_traffic(6, 65536)
    d, rsrc = bench.stored_rocprof(6, 65536, 20)
    if traffic is None or d is None:
        pytest.fail("the committed profiles do not match this build's step kernel: %s / %s" % (src, rsrc))
    with open(os.path.join(ROOT, src)) as f:
        rec = json.load(f)
    assert hashes[rec["kernel_name"]] == rec["isa_hash"]
