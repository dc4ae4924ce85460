"""Seeded synthetic batches for the BASELINE.json configs, as columns.

The wire bytes are produced from these columns by the product encoder (config 4). The
generators are numpy-vectorised, so that 10^7-10^8 records take seconds.

* f64 (configs 2, 4, 5): From::Update(Id(i), F64(x_i)) with i = 0..N-1 ascending, matching the
  order of Id::new (netidx-core/src/utils.rs:130-134). x_i is a SplitMix64 draw mapped to
  uniform(-1e6, 1e6), and 1 % of the values are specials: +-0, +-inf, quiet/signalling NaN
  with payloads, subnormals.
* mixed (config 3): the value tag is drawn as I64 25 %, F64 25 %, String 20 %, DateTime 15 %,
  Array 15 %.
  - String: byte length U[0,32]; the text is valid UTF-8, and 10 % of the strings contain
    multibyte code points.
  - DateTime: secs U[0, 4.1e9], ns U[0, 1e9).
  - Array: length U[0,8]; elements are F64 or I64, 50/50.
  - Ids are a seeded permutation of 0..N-1.
"""
import numpy as np

SEED_F64 = 0x5EED0002
SEED_MIXED = 0x5EED0003
SEED_8GPU = 0x5EED0005

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(n, seed, offset=0):
    """SplitMix64 stream, elements [offset, offset+n)."""
    with np.errstate(over="ignore"):
        z = (np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
             * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


SPECIALS = np.array([0x0000000000000000, 0x8000000000000000, 0x7FF0000000000000,
                     0xFFF0000000000000, 0x7FF8000000000001, 0x7FF4000000000123,
                     0xFFF8DEADBEEF0001, 0x0000000000000001, 0x800FFFFFFFFFFFFF,
                     0x000FFFFFFFFFFFFF], dtype=np.uint64)


def f64_columns(n, seed=SEED_F64, id_offset=0):
    """(ids u64[n], f64 bit patterns u64[n])."""
    r = splitmix64(n, seed, id_offset)
    x = (r >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53)) * 2e6 - 1e6
    bits = x.view(np.uint64).copy()
    sel = (r & np.uint64(127)) < np.uint64(1)  # ~0.8 %: ~1 % incl. the natural zeros
    k = (r >> np.uint64(7)) % np.uint64(len(SPECIALS))
    bits[sel] = SPECIALS[k[sel].astype(np.int64)]
    ids = np.arange(id_offset, id_offset + n, dtype=np.uint64)
    return ids, bits


class MixedColumns:
    """Host columns of a config-3 batch: rows + array children + a string heap."""

    def __init__(self, id, tag, fixed, aux, ctag, cfixed, caux, heap):
        self.id, self.tag, self.fixed, self.aux = id, tag, fixed, aux
        self.ctag, self.cfixed, self.caux, self.heap = ctag, cfixed, caux, heap

    @property
    def n(self):
        return len(self.id)


def mixed_columns(n, seed=SEED_MIXED):
    rng = np.random.default_rng(seed)
    ids = rng.permutation(n).astype(np.uint64)
    u = rng.random(n)
    tag = np.where(u < 0.25, 6, np.where(u < 0.50, 9, np.where(u < 0.70, 12,
                   np.where(u < 0.85, 10, 19)))).astype(np.uint8)
    fixed = np.zeros(n, np.uint64)
    aux = np.zeros(n, np.uint32)
    m = tag == 6
    fixed[m] = rng.integers(-(2**62), 2**62, int(m.sum()), dtype=np.int64).view(np.uint64)
    m = tag == 9
    fixed[m] = (rng.random(int(m.sum())) * 2e6 - 1e6).view(np.uint64)
    m = tag == 10
    k = int(m.sum())
    fixed[m] = rng.integers(0, 4_100_000_000, k, dtype=np.int64).view(np.uint64)
    aux[m] = rng.integers(0, 1_000_000_000, k, dtype=np.uint32)
    # strings: ASCII body, 10 % get multibyte code points at the front
    m = tag == 12
    ns = int(m.sum())
    slen = rng.integers(0, 33, ns).astype(np.int64)
    soff = np.zeros(ns, np.int64)
    soff[1:] = np.cumsum(slen)[:-1]
    heap = rng.integers(0x61, 0x7B, int(slen.sum()), dtype=np.uint8)  # a..z
    multi = (rng.random(ns) < 0.10)
    two = multi & (slen >= 2)
    heap[soff[two]] = 0xC3  # 'é' = C3 A9
    heap[soff[two] + 1] = 0xA9
    three = multi & (slen >= 5)
    heap[soff[three] + 2] = 0xE2  # '€' = E2 82 AC
    heap[soff[three] + 3] = 0x82
    heap[soff[three] + 4] = 0xAC
    fixed[m] = soff.astype(np.uint64)
    aux[m] = slen.astype(np.uint32)
    # arrays of 0..8 F64/I64 elements, children allocated in row order
    m = tag == 19
    na = int(m.sum())
    alen = rng.integers(0, 9, na).astype(np.int64)
    astart = np.zeros(na, np.int64)
    astart[1:] = np.cumsum(alen)[:-1]
    nch = int(alen.sum())
    ctag = np.where(rng.random(nch) < 0.5, 9, 6).astype(np.uint8)
    cfixed = np.where(ctag == 9, (rng.random(nch) * 2e6 - 1e6).view(np.uint64),
                      rng.integers(-(2**40), 2**40, nch, dtype=np.int64).view(np.uint64))
    caux = np.zeros(nch, np.uint32)
    fixed[m] = astart.astype(np.uint64)
    aux[m] = alen.astype(np.uint32)
    return MixedColumns(ids, tag, fixed, aux, ctag, cfixed.astype(np.uint64), caux, heap)


def mixed_columns_ctl(n, seed=SEED_MIXED, p_hb=0.01, p_long=0.01, long_len=200):
    """Config 3 as a live subscriber sees it: the mixed_columns rows with about p_long of the
    scalar rows turned into long_len-byte strings (two-byte length prefixes; every eighth holds
    multibyte code points) and about p_hb * n Heartbeats (From::Heartbeat, 02 05) between rows.
    Returns (MixedColumns, ctl_row, ctl_off, ctl_len, ctl_variant): the control spans point at
    one 02 05 appended to the heap."""
    m = mixed_columns(n, seed)
    rng = np.random.default_rng(seed + 7)
    long_rows = np.flatnonzero((rng.random(n) < p_long) & (m.tag != 19))
    k = len(long_rows)
    body = rng.integers(0x61, 0x7B, (k, long_len), dtype=np.uint8)
    body[::8, 100:103] = (0xE2, 0x82, 0xAC)  # '€'
    base = len(m.heap)
    m.tag[long_rows] = 12
    m.fixed[long_rows] = (base + long_len * np.arange(k)).astype(np.uint64)
    m.aux[long_rows] = long_len
    hb_off = base + k * long_len
    m.heap = np.concatenate([m.heap, body.reshape(-1), np.array([2, 5], np.uint8)])
    nh = int(round(n * p_hb))
    ctl_row = np.sort(rng.integers(0, n + 1, nh)).astype(np.uint64)
    ctl_off = np.full(nh, hb_off, np.uint64)
    ctl_len = np.full(nh, 2, np.uint32)
    ctl_variant = np.full(nh, 5, np.uint8)
    return m, ctl_row, ctl_off, ctl_len, ctl_variant


SEED_ARCHIVE = 0x5EED0006


def archive_columns(n, seed=SEED_ARCHIVE, p_unsub=0.05):
    """Rows of an archive batch (Vec<BatchItem>, netidx-archive logfile/mod.rs:150-205): the
    config-3 value mix with u32 Ids, and about p_unsub of the scalar rows turned into
    Event::Unsubscribed (tag 0x40)."""
    m = mixed_columns(n, seed)
    rng = np.random.default_rng(seed + 1)
    un = (rng.random(n) < p_unsub) & (m.tag != 19)
    m.tag[un] = 0x40
    m.fixed[un] = 0
    m.aux[un] = 0
    return m
