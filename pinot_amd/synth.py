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
    """A synthetic column generated on the device: BE dictionary bytes + BE forward bytes (device tensors) and the
    host-side dictionary (needed for predicate lowering, as the reference keeps its Dictionary on heap)."""
    spec: ColSpec
    num_docs: int
    cardinality: int
    bits: int
    dict_values: np.ndarray      # host, sorted unique
    dict_be: object              # torch uint8 (device)
    fwd_be: object               # torch uint8 (device)

    def meta_column(self) -> Column:
        """Host metadata + dictionary only (the forward index stays on the device)."""
        return Column(self.spec.name, self.spec.data_type, True, Dictionary(self.spec.data_type, self.dict_values),
                      self.num_docs, self.bits, False, self.num_docs)

    def host_column(self) -> Column:
        """Copy to host as a reference-format Column (for the CPU oracle / baseline)."""
        col = Column(self.spec.name, self.spec.data_type, True, Dictionary(self.spec.data_type, self.dict_values),
                     self.num_docs, self.bits, False, self.num_docs)
        col.fwd = self.fwd_be.cpu().numpy().tobytes()
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
