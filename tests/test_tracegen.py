"""Host restatement of the trace recipe (the device generator is checked
against it bit-for-bit in test_parity_gpu.py)."""
import numpy as np

import tracegen as tg


def test_philox_known_answer():
    # Random123 Philox4x32-10 known-answer vector (counter = key = 0)
    x = tg.philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in x] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_philox_known_answer_pi():
    x = tg.philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0)
    assert [int(v) for v in x] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_neg_log_unit_accuracy():
    u = np.concatenate([np.linspace(2**-53, 1.0, 100001), [2**-53, 0.5, 1.0, 0.7071067811865476]])
    ref = -np.log(u)
    got = tg.neg_log_unit(u)
    assert np.all(np.abs(got - ref) <= 4e-16 * np.maximum(1.0, np.abs(ref)))
    assert tg.neg_log_unit(np.array([1.0]))[0] == 0.0


def test_replication_shape_and_preconditions():
    rp = tg.make_replication(0x5EED0001, 0, 64, 10000)
    assert rp["arrive"].shape == (10000,) and rp["req"].dtype == np.int32
    assert np.all(np.diff(rp["arrive"]) >= 0)
    assert rp["init"].max() < rp["arrive"][0]
    assert np.all(rp["init"] >= rp["ul"])
    assert rp["req"].min() >= 1000 and rp["req"].max() <= 64000
    assert rp["dl"].min() >= 10**6 and rp["dl"].max() <= 10**9
    assert rp["mips"].tolist()[:5] == [1000, 2000, 3000, 4000, 1000]
    gaps = np.diff(rp["arrive"])
    es = tg.mean_service_seconds(rp["mips"])
    assert abs(gaps.mean() / (es / (64 * 0.8) * 1e12) - 1) < 0.05  # Poisson mean within 5 %


def test_replications_differ_and_are_reproducible():
    a = tg.make_replication(1, 0, 8, 100)
    b = tg.make_replication(1, 1, 8, 100)
    c = tg.make_replication(1, 0, 8, 100)
    assert not np.array_equal(a["req"], b["req"])
    for k in a:
        np.testing.assert_array_equal(a[k], c[k])
