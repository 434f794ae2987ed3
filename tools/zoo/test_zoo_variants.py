"""Parity tests of the rejected kernel variants kept in tools/zoo (KF_COUNT_VARIANT
selects one; variant 20 is known to be wrong on adversarial input and is
expected to fail).  The product's own tests are tests/test_gpu_parity.py."""
import numpy as np
import pytest

import gen
from test_gpu_parity import _k1x_wave_ranges, check_against_oracle, counter, run_batch, torch_dev  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [18, 19, 21, 22, 23, pytest.param(20, marks=pytest.mark.xfail(
    reason="variant 20 checks returns every other iteration: a counter grown only in unchecked iterations "
           "passes 0xFFFF", strict=True))])
def test_zoo_k7_unchecked_iterations_adversarial(torch_dev, oracle, monkeypatch, variant):
    monkeypatch.setenv("KF_COUNT_VARIANT", str(variant))
    monkeypatch.delenv("KF_WAVE_WEIGHTS", raising=False)
    rng = np.random.default_rng(99)
    L = 80_000_000
    head = b">adv\n"
    arr = np.frombuffer(b"CGT", np.uint8)[rng.integers(0, 3, L)].copy()
    grid = counter(7, torch_dev).launch_info()[0]
    total = (L + 15) // 16 * 16
    for lo, hi in _k1x_wave_ranges(total, grid):
        c0 = lo & ~15
        i = 1
        while c0 + 3072 * (i + 1) <= hi:
            arr[c0 + 3072 * i: c0 + 3072 * (i + 1)] = ord("A")
            i += 2
    arr[: len(head)] = np.frombuffer(head, np.uint8)
    pos = np.arange(len(head), L)
    arr[pos[(pos - len(head)) % 81 == 80]] = 10
    blobs = [arr.tobytes()]
    counts, totals = run_batch(blobs, 7, torch_dev)
    check_against_oracle(oracle, blobs, 7, counts, totals, tag=f"adv-v{variant}")


@pytest.mark.parametrize("k", [9, 10])
def test_bucket_kernel_agrees_with_other_large_k_paths(torch_dev, monkeypatch, k):
    """k=9: bucket vs multi-pass LDS; k=10: bucket vs global atomics (KF_BUCKET_MIN_K)."""
    import torch
    from kf2vecfsw_amd import counter as C
    db = C.synth_device_batch(40, 700_000, seed0=5, n_period=3, device=torch_dev)
    kc = counter(k, torch_dev)
    out = {}
    for thr in (9, 13):
        monkeypatch.setenv("KF_BUCKET_MIN_K", str(thr))
        c, t = kc.count(db)
        torch.cuda.synchronize()
        out[thr] = (c.clone(), t.clone())
    assert torch.equal(out[9][0], out[13][0]) and torch.equal(out[9][1], out[13][1])



@pytest.mark.parametrize("variant", [0, 1, 2, 8, 9])
@pytest.mark.parametrize("k", [3, 5, 7, 8])
def test_count_kernel_variants_match_oracle(torch_dev, oracle, monkeypatch, variant, k):
    """The other shapes of the count kernel (KF_COUNT_VARIANT: 512-thread, the
    1024-thread forward histogram K1 that k=7 used before K1w, 6-deep prefetch ring,
    dynamic-chunk kernels with 4- and 6-deep rings) on ragged FASTA."""
    monkeypatch.setenv("KF_COUNT_VARIANT", str(variant))
    rng = np.random.default_rng(300 + 10 * variant + k)
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 200000)), max_records=5, n_rate=0.002, lower=0.05,
                              crlf_rate=0.05) for _ in range(20)]
    counts, totals = run_batch(blobs, k, torch_dev)
    check_against_oracle(oracle, blobs, k, counts, totals, tag=f"v{variant}")



@pytest.mark.parametrize("variant", [5, 6, 7, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23])
def test_k7_kernel_variants_agree(torch_dev, oracle, monkeypatch, variant):
    """k=7 pair kernels (KF_COUNT_VARIANT 5, 6, 7: self-contained chunks, prefetch
    ring 6 / 4 / 8; 10, 11: static wave ranges, ring 6 / 8; 12, 13: 32-byte lanes,
    ring 2 / 3) on ragged FASTA, like
    the default forward-histogram kernel."""
    monkeypatch.setenv("KF_COUNT_VARIANT", str(variant))
    rng = np.random.default_rng(500 + variant)
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 300000)), max_records=5, n_rate=0.002, lower=0.05,
                              crlf_rate=0.05, poly_rate=0.01) for _ in range(20)]
    counts, totals = run_batch(blobs, 7, torch_dev)
    check_against_oracle(oracle, blobs, 7, counts, totals, tag=f"v{variant}")



@pytest.mark.parametrize("frac,unit", [("0", "1"), ("0.5", "3"), ("1", "2"), ("0.85", "2"), ("0.9", "64")])
def test_k7_claimed_units(torch_dev, oracle, monkeypatch, frac, unit):
    """Variant 22 (K1x whose waves claim the last part of each piece in units
    from a per-workgroup ticket): every static/claimed split, unit sizes from one
    3 KiB iteration to 64, low-complexity genomes whose u16 drains happen inside
    claimed units, and repeated launches (the tickets continue across launches)."""
    monkeypatch.setenv("KF_COUNT_VARIANT", "22")
    monkeypatch.setenv("KF_DYN_FRAC", frac)
    monkeypatch.setenv("KF_DYN_UNIT", unit)
    rng = np.random.default_rng(777 + int(float(frac) * 100) + int(unit))
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 1_500_000)), max_records=4, n_rate=0.002, lower=0.05,
                              crlf_rate=0.02, poly_rate=0.01) for _ in range(24)]
    blobs.append(b">polyA\n" + gen.wrap(np.frombuffer(b"A" * 6_000_000, np.uint8), 80))
    blobs.append(b">ac\n" + gen.wrap(np.frombuffer(b"AC" * 2_000_000, np.uint8), 61))
    for rep in range(2):
        counts, totals = run_batch(blobs, 7, torch_dev)
        check_against_oracle(oracle, blobs, 7, counts, totals, tag=f"claim-{frac}-{unit}-{rep}")



def test_k7_stealing_repeated_launches(torch_dev, oracle, monkeypatch):
    """Variant 23 (waves claim their own iterations from the front while idle
    waves take back halves): genomes of every size class in one batch, several
    launches in a row (the range words persist between launches, tagged by piece)."""
    monkeypatch.setenv("KF_COUNT_VARIANT", "23")
    rng = np.random.default_rng(2323)
    blobs = [gen.random_fasta(rng, int(rng.choice([0, 100, 5000, 300_000, 3_000_000])), max_records=6, n_rate=0.002,
                              lower=0.05, crlf_rate=0.01, poly_rate=0.01) for _ in range(40)]
    blobs.append(b">polyA\n" + gen.wrap(np.frombuffer(b"A" * 8_000_000, np.uint8), 80))
    for rep in range(3):
        counts, totals = run_batch(blobs, 7, torch_dev)
        check_against_oracle(oracle, blobs, 7, counts, totals, tag=f"steal-{rep}")


