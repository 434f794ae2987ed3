"""GPU parity of the device FASTA record index (kf_index_fasta) against the host
index (kf_index_records) and, through kf_count_batch, against the oracle."""
import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev(native):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests need an MI355X")
    return torch.device("cuda:0")


def excluded_mask(pairs: np.ndarray, n: int) -> np.ndarray:
    m = np.zeros(n, dtype=bool)
    for s, e in pairs.reshape(-1, 2):
        m[int(s): int(e)] = True
    return m


def corpus(rng):
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 40000)), n_rate=0.01, lower=0.05, crlf_rate=0.2)
             for _ in range(12)]
    blobs += [b"", b">only\n", b">a\n>b\n>c\nACGT\n", b"ACGT>ACGT\n>h>x\nGG>\n", b">no newline at the end",
              b"junk before\n>r1\nACGTACGT\n\n\n>r2 x>y\nTTTT", b">" * 50 + b"\nACGT\n", b"\n>\n>\n\n>\nA"]
    return blobs


def test_device_index_matches_host(torch_dev):
    """The same excluded bytes as the host index on ragged multi-record FASTA:
    headers with '>' inside, consecutive header lines, CRLF, a header at the very
    end without '\\n', bytes before the first header, genomes that end without a
    newline right before the next genome's '>'."""
    import torch
    from kf2vecfsw_amd import counter as C
    rng = np.random.default_rng(41)
    blobs = corpus(rng)
    hb_host = C.pack_genomes(blobs)
    hb = C.HostBatch(hb_host.data, hb_host.off, None, hb_host.names)
    db = C.to_device(hb, torch_dev)
    torch.cuda.synchronize()
    n = int(hb.off[-1])
    # the host merges header lines that follow each other (their '\n' inside the
    # merged range); newlines are transparent either way, so compare the rest
    nl = hb_host.data.numpy()[:n] == 10
    got = excluded_mask(db.excl[: 2 * db.n_excl].cpu().numpy(), n)
    exp = excluded_mask(hb_host.excl, n)
    assert np.array_equal(got & ~nl, exp & ~nl)
    pairs = db.excl[: 2 * db.n_excl].cpu().numpy()
    assert np.all(np.diff(pairs) >= 0)   # sorted, disjoint
    # genomes packed without '\n' padding between them: the next genome's '>' starts a header
    tight = [b"ACGTACGTACGTACGT", b">x\nACGT\n", b"CCCCCCCCCCCCCCCC", b">y\nGG"]
    off = np.cumsum([0] + [len(b) for b in tight]).astype(np.uint64)
    data = torch.full((int(off[-1]) + 16,), 10, dtype=torch.uint8)
    data.numpy()[: int(off[-1])] = np.frombuffer(b"".join(tight), np.uint8)
    db = C.to_device(C.HostBatch(data, off, None, ["t"] * 4), torch_dev)
    pairs = db.excl[: 2 * db.n_excl].cpu().numpy().tolist()
    assert pairs == [16, 18, 40, 42], pairs


@pytest.mark.parametrize("k", [7, 11])
def test_device_index_counts_equal_oracle(torch_dev, oracle, k):
    """kf_count_batch over the device index == the oracle, genome by genome."""
    import torch
    from kf2vecfsw_amd import counter as C
    rng = np.random.default_rng(43 + k)
    blobs = corpus(rng)
    hb_host = C.pack_genomes(blobs)
    db = C.to_device(C.HostBatch(hb_host.data, hb_host.off, None, hb_host.names), torch_dev)
    cnt, tot = C.KmerCounter(k, torch_dev).count(db)
    torch.cuda.synchronize()
    c = C.counts_to_numpy(cnt)
    t = tot.cpu().numpy()
    for i, b in enumerate(blobs):
        oc, ot = oracle.count(b, k)
        assert int(t[i]) == ot, (i, int(t[i]), ot)
        assert np.array_equal(c[i], oc), i


def test_device_index_table_regrows(torch_dev):
    """More header lines than the first table holds (one per 4 bytes): the index
    is run again with a table of the reported size."""
    import torch
    from kf2vecfsw_amd import counter as C
    blob = b"".join(b">%d\nA\n" % i for i in range(30000))
    hb_host = C.pack_genomes([blob])
    db = C.to_device(C.HostBatch(hb_host.data, hb_host.off, None, ["x"]), torch_dev)
    torch.cuda.synchronize()
    assert db.n_excl == 30000
    n = int(hb_host.off[-1])
    nl = hb_host.data.numpy()[:n] == 10
    got = excluded_mask(db.excl[: 2 * db.n_excl].cpu().numpy(), n)
    assert np.array_equal(got & ~nl, excluded_mask(hb_host.excl, n) & ~nl)
