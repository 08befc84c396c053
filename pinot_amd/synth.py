"""Deterministic synthetic segments for the benchmark configurations (BASELINE.md / SURVEY.md §8(d)).

Every value is a pure function of (seed, column, global row): a 32-bit murmur-style finalizer of the row index
salted per column, mapped to [lo, lo + range) by multiply-shift.  So each GPU (or the CPU) regenerates exactly its
own segments, and the numpy path (CPU, small tests) and the torch path (device, full size) produce identical bytes.

Segments are written in Pinot's own format, as SegmentColumnarIndexCreator / SegmentDictionaryCreator would:
sorted unique dictionary of the values present in the segment, bitsPerElement =
PinotDataBitSet.getNumBitsPerValue(cardinality - 1), dictIds bit-packed MSB-first big-endian
(FixedBitSVForwardIndexWriter.java:42-44).  Test/bench data only: nothing here is on the query path.
"""
from __future__ import annotations

import zlib
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from .segment import Column, Dictionary, ImmutableSegment, num_bits_per_value, pack_bits

SEED = 42  # BenchmarkQueries.java:188
M32 = 0xFFFFFFFF


@dataclass(frozen=True)
class ColSpec:
    name: str
    lo: int
    range: int
    data_type: str = "INT"


# Config 2 (north star): AdAnalytics, SURVEY.md §8(d)
ADANALYTICS = [
    ColSpec("daysSinceEpoch", 17900, 365),
    ColSpec("accountId", 0, 1_000_000),
    ColSpec("clicks", 0, 1000),
    ColSpec("impressions", 0, 100_000),
]
ADANALYTICS_ROWS_PER_SEGMENT = 7_812_500
ADANALYTICS_SEGMENTS = 128


def adanalytics_query(num_ids: int = 1000) -> str:
    """Config 2 query: 90-day range (24.7 % of days) AND accountId IN (num_ids ids) GROUP BY daysSinceEpoch."""
    ids = ", ".join(str((i * 7919 + 13) % 1_000_000) for i in range(num_ids))
    return ("SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics "
            f"WHERE daysSinceEpoch BETWEEN 18000 AND 18089 AND accountId IN ({ids}) "
            "GROUP BY daysSinceEpoch ORDER BY daysSinceEpoch LIMIT 400")


# Config 3: SSB-style lineorder; dates as day numbers (8035 = 1992-01-01), 2 557 days
SSB_LINEORDER = [
    ColSpec("lo_orderdate", 8035, 2557),
    ColSpec("lo_discount", 0, 11),
    ColSpec("lo_quantity", 1, 50),
    ColSpec("lo_extendedprice", 90_000, 1 << 20),
]
SSB_SEGMENTS_PER_GPU = 96  # 768 segments of 7 812 500 rows = 6 B rows over 8 GPUs


def ssb_q11_query() -> str:
    """Config 3 query (SSB Q1.1 shape): one year of orders, discount 1..3, quantity < 25."""
    return ("SELECT SUM(lo_extendedprice * lo_discount) FROM lineorder "
            "WHERE lo_orderdate BETWEEN 8035 AND 8399 AND lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25")


# Config 4: high-cardinality group-by: 10 M users x 1 000 items, 128 segments of 7 812 500 rows
def highcard_specs(users: int = 10_000_000, items: int = 1000) -> List[ColSpec]:
    return [ColSpec("userId", 0, users), ColSpec("itemId", 0, items)]


HIGHCARD = highcard_specs()


def highcard_query(limit: int = 100) -> str:
    """Config 4 query: distinct items per user, top users (a total order: userId breaks DISTINCTCOUNT ties)."""
    return ("SELECT userId, DISTINCTCOUNT(itemId) FROM events GROUP BY userId "
            f"ORDER BY DISTINCTCOUNT(itemId) DESC, userId LIMIT {limit}")


# Config 5: index path: 2 B rows = 256 segments (32 per GPU at N = 8).  sortedCol is sorted within
# every segment over 100 000 values (sorted index: 800 KB of (start, end) pairs per segment); inv1..inv4 carry bitmap
# inverted indexes; mvTags is multi-value (1-7 values per doc, 4 on average, over 1 000 tags).
INDEX_SORTED = ColSpec("sortedCol", 0, 100_000)
INDEX_INVERTED = [ColSpec("inv1", 0, 10), ColSpec("inv2", 0, 100), ColSpec("inv3", 0, 1000), ColSpec("inv4", 0, 10_000)]
INDEX_MV = ColSpec("mvTags", 0, 1000)
INDEX_SEGMENTS_PER_GPU = 32


def index_query() -> str:
    """Config 5 query: a 40 % sortedCol range AND (inv1 = x OR inv2 IN 20 of 100) AND inv3 <> y AND inv4 IN 2 000 of
    10 000 -> about 2.2 % of the docs; COUNT(*) and COUNTMV over the multi-value column."""
    ids = ", ".join(str(i * 5 + 1) for i in range(2000))
    inv2 = ", ".join(str(i * 5) for i in range(20))
    return ("SELECT COUNT(*), COUNTMV(mvTags) FROM idx WHERE sortedCol BETWEEN 20000 AND 59999 "
            f"AND (inv1 = 3 OR inv2 IN ({inv2})) AND inv3 <> 7 AND inv4 IN ({ids})")


def index_values_np(seg_index: int, n: int) -> Dict[str, object]:
    """Values of one config-5 segment (numpy; identical to the device path)."""
    row0 = seg_index * n
    out = {"sortedCol": (np.arange(n, dtype=np.int64) * INDEX_SORTED.range) // n}
    for c in INDEX_INVERTED:
        out[c.name] = values_np(c, row0, n)
    lengths, flat = mv_values_np(seg_index, n)
    out["mvTags"] = np.split(flat, np.cumsum(lengths)[:-1])
    return out


def mv_values_np(seg_index: int, n: int):
    """mvTags: per doc 1 + (hash % 7) values, each a hash of the value's global position."""
    row0 = seg_index * n
    lengths = 1 + (hash32_np(np.arange(row0, row0 + n, dtype=np.uint64), column_salt("mvTags.len")) % np.uint64(7))
    lengths = lengths.astype(np.int64)
    v0 = int(seg_index) * n * 8
    flat = values_np(INDEX_MV, v0, int(lengths.sum()))
    return lengths, flat


def make_index_segment_np(seg_index: int, n: int) -> ImmutableSegment:
    return ImmutableSegment.create(f"idx_{seg_index}", index_values_np(seg_index, n),
                                   {"sortedCol": "INT", "inv1": "INT", "inv2": "INT", "inv3": "INT", "inv4": "INT",
                                    "mvTags": "INT"}, inverted=[c.name for c in INDEX_INVERTED])


# Config 1: pinot-tools QuickStart baseballStats (CPU-reference scale).  The data CSV is not in the reference checkout
# (.MISSING_LARGE_BLOBS), so rows follow the schema (pinot-tools/.../baseballStats/baseballStats_schema.json: 5 STRING /
# INT dimensions, 20 INT metrics) with plausible ranges; inverted indexes on playerID and teamID as its table config.
BASEBALL_METRICS = ["playerStint", "numberOfGames", "numberOfGamesAsBatter", "AtBatting", "runs", "hits", "doules",
                    "tripples", "homeRuns", "runsBattedIn", "stolenBases", "caughtStealing", "baseOnBalls", "strikeouts",
                    "intentionalWalks", "hitsByPitch", "sacrificeHits", "sacrificeFlies", "groundedIntoDoublePlays",
                    "G_old"]


def baseball_segment(rows: int = 97_889, players: int = 18_000, seed: int = SEED) -> ImmutableSegment:
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, players, rows)
    first = np.array(["John", "Bill", "Joe", "Jim", "Frank", "George", "Tom", "Charlie", "Ed", "Harry", "Mike",
                      "Bob", "Dave", "Fred", "Jack", "Al", "Pete", "Sam", "Walter", "Lou"], dtype=object)
    last = np.array([f"Player{i:05d}" for i in range(players // 3)], dtype=object)
    # names collide across players (different playerIDs, one playerName), as in the real table
    names = np.array([f"{first[i % len(first)]} {last[(i * 7919) % len(last)]}" for i in range(players)], dtype=object)
    teams = np.array([f"T{i:03d}" for i in range(149)], dtype=object)
    data = {"playerID": np.array([f"p{i:06d}" for i in range(players)], dtype=object)[pid],
            "playerName": names[pid],
            "yearID": rng.integers(1871, 2014, rows),
            "teamID": teams[rng.integers(0, len(teams), rows)],
            "league": np.array(["AL", "NL", "AA", "UA", "FL", "PL"], dtype=object)[rng.integers(0, 6, rows)]}
    hi = {"playerStint": 5, "numberOfGames": 165, "numberOfGamesAsBatter": 165, "AtBatting": 716, "runs": 192,
          "hits": 262, "doules": 67, "tripples": 36, "homeRuns": 73, "runsBattedIn": 191, "stolenBases": 138,
          "caughtStealing": 42, "baseOnBalls": 232, "strikeouts": 223, "intentionalWalks": 120, "hitsByPitch": 51,
          "sacrificeHits": 67, "sacrificeFlies": 19, "groundedIntoDoublePlays": 36, "G_old": 165}
    for m in BASEBALL_METRICS:
        data[m] = (rng.integers(0, hi[m] + 1, rows) * rng.random(rows) ** 2).astype(np.int64)
    schema = {"playerID": "STRING", "playerName": "STRING", "yearID": "INT", "teamID": "STRING", "league": "STRING"}
    schema.update({m: "INT" for m in BASEBALL_METRICS})
    return ImmutableSegment.create("baseballStats_OFFLINE_0", data, schema, inverted=["playerID", "teamID"])


# pinot-tools Quickstart.java:185-213 queries, LIMIT 10 with playerName as the tie-break of equal sums
BASEBALL_QUERIES = [
    "SELECT COUNT(*) FROM baseballStats",
    "SELECT playerName, SUM(runs) FROM baseballStats GROUP BY playerName ORDER BY SUM(runs) DESC, playerName LIMIT 10",
    "SELECT playerName, SUM(runs) FROM baseballStats WHERE yearID = 2000 GROUP BY playerName "
    "ORDER BY SUM(runs) DESC, playerName LIMIT 10",
    "SELECT playerName, SUM(runs) FROM baseballStats WHERE yearID >= 2000 GROUP BY playerName "
    "ORDER BY SUM(runs) DESC, playerName LIMIT 10",
    "SELECT teamID, COUNT(*), SUM(homeRuns), MAX(hits), AVG(runs) FROM baseballStats WHERE teamID IN ('T001', 'T017', "
    "'T100') OR league = 'NL' GROUP BY teamID ORDER BY SUM(homeRuns) DESC, teamID LIMIT 10",
    "SELECT league, DISTINCTCOUNT(playerID), SUM(runs) FROM baseballStats WHERE playerID <> 'p000007' GROUP BY league",
]


def column_salt(name: str) -> int:
    return (zlib.crc32(name.encode()) ^ (SEED * 0x9E3779B1)) & M32


# ----------------------------------------------------------------------------------------- numpy (CPU)

def hash32_np(rows: np.ndarray, salt: int) -> np.ndarray:
    h = (rows.astype(np.uint64) * np.uint64(0x9E3779B1) + np.uint64(salt)) & np.uint64(M32)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(M32)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(M32)
    h ^= h >> np.uint64(16)
    return h


def values_np(spec: ColSpec, row0: int, n: int) -> np.ndarray:
    rows = np.arange(row0, row0 + n, dtype=np.uint64)
    h = hash32_np(rows, column_salt(spec.name))
    return (np.int64(spec.lo) + ((h * np.uint64(spec.range)) >> np.uint64(32)).astype(np.int64))


def make_segment_np(specs: Sequence[ColSpec], seg_index: int, rows_per_segment: int,
                    name: Optional[str] = None) -> ImmutableSegment:
    """One synthetic segment in Pinot format (CPU)."""
    row0 = seg_index * rows_per_segment
    data = {s.name: values_np(s, row0, rows_per_segment) for s in specs}
    return ImmutableSegment.create(name or f"synth_{seg_index}", data, {s.name: s.data_type for s in specs})


# ----------------------------------------------------------------------------------------- torch (device)

def hash32_torch(rows, salt: int):
    import torch
    h = (rows * 0x9E3779B1 + salt) & M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    h = h ^ (h >> 16)
    return h


def pack_bits_torch(ids, b: int):
    """Device bit-packing of non-negative int64 ids (< 2^b) into the reference's big-endian byte stream."""
    import torch
    n = ids.numel()
    nbytes = (n * b + 7) // 8
    nwords = (n * b + 31) // 32 + 1
    p = torch.arange(n, device=ids.device, dtype=torch.int64) * b
    w = p >> 5
    off = p & 31
    s1 = 32 - off - b
    hi = torch.where(s1 >= 0, ids << s1.clamp(min=0), ids >> (-s1).clamp(min=0))
    spill = (off + b) > 32
    lo = torch.where(spill, (ids << (64 - off - b).clamp(min=0, max=63)) & M32, torch.zeros_like(ids))
    words = torch.zeros(nwords + 1, dtype=torch.int64, device=ids.device)
    words.index_add_(0, w, hi)
    words.index_add_(0, w + 1, lo)
    be = torch.stack([(words >> 24) & 255, (words >> 16) & 255, (words >> 8) & 255, words & 255], dim=1)
    return be.to(torch.uint8).reshape(-1)[:nbytes].contiguous()


def be_int32_torch(v):
    import torch
    v = v & M32
    return torch.stack([(v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255], dim=1).to(torch.uint8).reshape(-1)


@dataclass
class DeviceColumn:
    """A synthetic column generated on the device: BE dictionary bytes + BE forward bytes (+ the bitmap inverted index
    bytes) as device tensors and the host-side dictionary (needed for predicate lowering, as the reference keeps its
    Dictionary on heap).  kind: "sv" (bit-packed), "sorted" ((start, end) pairs), "mv" (FixedBitMVForwardIndexWriter)."""
    spec: ColSpec
    num_docs: int
    cardinality: int
    bits: int
    dict_values: np.ndarray      # host, sorted unique
    dict_be: object              # torch uint8 (device)
    fwd_be: object               # torch uint8 (device)
    kind: str = "sv"
    num_values: int = 0          # MV: totalNumberOfEntries
    max_mv: int = 0
    inv_be: object = None        # torch uint8 (device): BitmapInvertedIndexWriter layout, or None

    def _column(self) -> Column:
        return Column(self.spec.name, self.spec.data_type, self.kind != "mv",
                      Dictionary(self.spec.data_type, self.dict_values), self.num_docs, self.bits,
                      self.kind == "sorted", self.num_values or self.num_docs, self.max_mv)

    def meta_column(self) -> Column:
        """Host metadata + dictionary only (the indexes stay on the device); `inverted` marks an inverted index."""
        col = self._column()
        if self.inv_be is not None:
            col.inverted = b"<device>"
        return col

    def host_column(self) -> Column:
        """Copy to host as a reference-format Column (for the CPU oracle / baseline)."""
        col = self._column()
        col.fwd = self.fwd_be.cpu().numpy().tobytes()
        if self.inv_be is not None:
            col.inverted = self.inv_be.cpu().numpy().tobytes()
        return col


def make_columns_torch(specs: Sequence[ColSpec], seg_index: int, rows_per_segment: int, device) -> List[DeviceColumn]:
    import torch
    row0 = seg_index * rows_per_segment
    rows = torch.arange(row0, row0 + rows_per_segment, dtype=torch.int64, device=device)
    out = []
    for s in specs:
        h = hash32_torch(rows, column_salt(s.name))
        v = s.lo + ((h * s.range) >> 32)
        uniq, inv = torch.unique(v, sorted=True, return_inverse=True)
        card = uniq.numel()
        b = num_bits_per_value(card - 1)
        out.append(DeviceColumn(s, rows_per_segment, card, b, uniq.cpu().numpy().astype(np.int32),
                                be_int32_torch(uniq), pack_bits_torch(inv.to(torch.int64), b)))
    return out


# ----------------------------------------------------------------------------------------- config 5 (device)

def _le_bytes(x, nbytes: int):
    """Little-endian bytes of int64 tensor x: [n, nbytes] uint8."""
    import torch
    sh = torch.arange(nbytes, device=x.device, dtype=torch.int64) * 8
    return ((x.unsqueeze(1) >> sh) & 255).to(torch.uint8)


def inverted_index_torch(ids, card: int, num_docs: int):
    """BitmapInvertedIndexWriter bytes ((card + 1) BE uint32 offsets, then per dictId a portable RoaringBitmap of its
    docs) built on the device for a column whose every dictId occurs.  Containers are arrays (<= 4 096 docs) or
    bitmaps, as RoaringBitmap chooses without runOptimize gains (checked: no container here would shrink as runs)."""
    import torch
    dev = ids.device
    n = ids.numel()
    docs = torch.arange(n, device=dev, dtype=torch.int64)
    sv, order = torch.sort(ids * (1 << 32) + docs)
    sdoc = sv & 0xFFFFFFFF
    sval = sv >> 32
    nkeys = (num_docs + 65535) >> 16
    cid = sval * nkeys + (sdoc >> 16)
    cu, ccount = torch.unique_consecutive(cid, return_counts=True)
    nc = cu.numel()
    cval, ckey = cu // nkeys, cu % nkeys
    # run containers would be chosen when 2 + 4 * runs < plain size (RoaringBitmap.runOptimize)
    cstart = torch.cumsum(ccount, 0) - ccount
    entry_c = torch.repeat_interleave(torch.arange(nc, device=dev), ccount)
    low = sdoc & 0xFFFF
    brk = torch.ones(n, dtype=torch.int64, device=dev)
    brk[1:] = ((low[1:] - low[:-1]) != 1).to(torch.int64) | (entry_c[1:] != entry_c[:-1]).to(torch.int64)
    runs = torch.zeros(nc, dtype=torch.int64, device=dev).index_add_(0, entry_c, brk)
    is_bm = ccount > 4096
    psize = torch.where(is_bm, torch.full_like(ccount, 8192), 2 * ccount)
    if bool(((2 + 4 * runs) < psize).any()):
        raise ValueError("a run container would be smaller: not generated on the device")
    nv = torch.bincount(cval, minlength=card)
    if bool((nv == 0).any()):
        raise ValueError("every dictId must occur")
    vstart_c = torch.cumsum(nv, 0) - nv                      # first container of each value
    rank_c = torch.arange(nc, device=dev) - vstart_c[cval]   # container index within its bitmap
    hdr = 8 + 8 * nv                                         # cookie + size + (key, card-1) pairs + offsets
    pay = torch.zeros(card, dtype=torch.int64, device=dev).index_add_(0, cval, psize)
    size_v = hdr + pay
    base = 4 * (card + 1)
    off_v = base + torch.cumsum(size_v, 0) - size_v          # absolute position of each bitmap in the file
    total = base + int(size_v.sum())
    out = torch.zeros(total, dtype=torch.uint8, device=dev)
    head = torch.cat([off_v, torch.tensor([total], device=dev)])
    out[:base] = torch.stack([(head >> 24) & 255, (head >> 16) & 255, (head >> 8) & 255, head & 255],
                             dim=1).to(torch.uint8).reshape(-1)
    p = off_v.unsqueeze(1) + torch.arange(8, device=dev)
    out[p.reshape(-1)] = torch.cat([_le_bytes(torch.full_like(nv, 12346), 4), _le_bytes(nv, 4)], dim=1).reshape(-1)
    pc = off_v[cval] + 8 + 4 * rank_c
    out[(pc.unsqueeze(1) + torch.arange(4, device=dev)).reshape(-1)] = \
        torch.cat([_le_bytes(ckey, 2), _le_bytes(ccount - 1, 2)], dim=1).reshape(-1)
    # payload offsets (from the bitmap's start): header, then the payloads of the earlier containers of the value
    pexcl = torch.cumsum(psize, 0) - psize
    prel = hdr[cval] + pexcl - pexcl[vstart_c[cval]]
    po = off_v[cval] + 8 + 4 * nv[cval] + 4 * rank_c
    out[(po.unsqueeze(1) + torch.arange(4, device=dev)).reshape(-1)] = _le_bytes(prel, 4).reshape(-1)
    pay_at = off_v[cval] + prel                              # absolute payload position of each container
    arr = ~is_bm[entry_c]
    erank = torch.arange(n, device=dev) - cstart[entry_c]
    pa = pay_at[entry_c][arr] + 2 * erank[arr]
    out[(pa.unsqueeze(1) + torch.arange(2, device=dev)).reshape(-1)] = _le_bytes(low[arr], 2).reshape(-1)
    bm = ~arr
    if bool(bm.any()):
        pb = pay_at[entry_c][bm] + (low[bm] >> 3)
        acc = torch.zeros(total, dtype=torch.int32, device=dev)
        acc.index_add_(0, pb, (1 << (low[bm] & 7)).to(torch.int32))
        out |= acc.to(torch.uint8)
    return out


def make_index_columns_torch(seg_index: int, n: int, device) -> List[DeviceColumn]:
    """One config-5 segment on the device, in the reference's byte layouts (same values as index_values_np)."""
    import torch
    out = []
    row0 = seg_index * n
    # sortedCol: value = dictId (every value of [0, 100 000) occurs when n >= 100 000), (start, end) pairs
    sv = (torch.arange(n, device=device, dtype=torch.int64) * INDEX_SORTED.range) // n
    uniq, cnt = torch.unique_consecutive(sv, return_counts=True)
    ends = torch.cumsum(cnt, 0) - 1
    starts = ends - cnt + 1
    card = uniq.numel()
    pairs = torch.stack([starts, ends], dim=1).reshape(-1)
    out.append(DeviceColumn(INDEX_SORTED, n, card, num_bits_per_value(card - 1), uniq.cpu().numpy().astype(np.int32),
                            be_int32_torch(uniq), be_int32_torch(pairs), kind="sorted"))
    rows = torch.arange(row0, row0 + n, dtype=torch.int64, device=device)
    for s in INDEX_INVERTED:
        h = hash32_torch(rows, column_salt(s.name))
        v = s.lo + ((h * s.range) >> 32)
        uq, inv = torch.unique(v, sorted=True, return_inverse=True)
        c = uq.numel()
        b = num_bits_per_value(c - 1)
        out.append(DeviceColumn(s, n, c, b, uq.cpu().numpy().astype(np.int32), be_int32_torch(uq),
                                pack_bits_torch(inv.to(torch.int64), b), inv_be=inverted_index_torch(inv, c, n)))
    lengths = 1 + (hash32_torch(rows, column_salt("mvTags.len")) % 7)
    nvals = int(lengths.sum())
    vrows = torch.arange(seg_index * n * 8, seg_index * n * 8 + nvals, dtype=torch.int64, device=device)
    v = INDEX_MV.lo + ((hash32_torch(vrows, column_salt(INDEX_MV.name)) * INDEX_MV.range) >> 32)
    uq, inv = torch.unique(v, sorted=True, return_inverse=True)
    c = uq.numel()
    b = num_bits_per_value(c - 1)
    starts = torch.cumsum(lengths, 0) - lengths
    dpc = int(np.ceil(np.float32(2048) / np.float32(nvals // n)))  # FixedBitMVForwardIndexReader.java:61
    nchunks = (n + dpc - 1) // dpc
    chunk_offsets = be_int32_torch(starts[::dpc][:nchunks])
    nbytes = (nvals + 7) // 8
    bits = torch.zeros(nbytes, dtype=torch.int32, device=device)
    bits.index_add_(0, starts >> 3, (128 >> (starts & 7)).to(torch.int32))  # MSB-first (PinotDataBitSet)
    fwd = torch.cat([chunk_offsets, bits.to(torch.uint8), pack_bits_torch(inv.to(torch.int64), b)])
    out.append(DeviceColumn(INDEX_MV, n, c, b, uq.cpu().numpy().astype(np.int32), be_int32_torch(uq), fwd, kind="mv",
                            num_values=nvals, max_mv=int(lengths.max())))
    return out
