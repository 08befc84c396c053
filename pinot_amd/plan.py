"""GpuPlanMaker: QueryContext + segments -> lowered pg_plan (C ABI), and the value-keyed results.

Host-side mirror of the reference's planning for the hot path:
  * predicate lowering to dictId space per segment -- PredicateEvaluatorProvider.getPredicateEvaluator
    (operator/filter/predicate/PredicateEvaluatorProvider.java:38-90) with the dictionary-based
    EQ / NOT_EQ / IN / NOT_IN / RANGE evaluators (EqualsPredicateEvaluatorFactory.java:85-110,
    NotEqualsPredicateEvaluatorFactory.java:85-, InPredicateEvaluatorFactory.java:153-199,
    NotInPredicateEvaluatorFactory.java:153-, RangePredicateEvaluatorFactory.java:115-210) and their
    isAlwaysTrue / isAlwaysFalse shortcuts;
  * leaf operator choice -- FilterOperatorUtils.getLeafFilterOperator (operator/filter/FilterOperatorUtils.java:45-85):
    always-false -> Empty, always-true -> MatchAll, sorted -> SortedIndex, RANGE + range index -> RangeIndex,
    inverted (non-RANGE) -> Bitmap, else scan;
  * group keys -- table-global key ids so that the device merges segments by VALUE the way
    GroupByOrderByCombineOperator merges Key(Object[]) (operator/combine/GroupByOrderByCombineOperator.java:176-183).
"""
from __future__ import annotations

import copy
import ctypes as C
import itertools
import math
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .query import (UNBOUNDED, Aggregation, Expr, FilterContext, Predicate, QueryContext, SelectItem,
                    filter_str)
from .segment import Column, Dictionary, ImmutableSegment

MAX_VALUE_OFFSET_KEYS = 1 << 26   # integer key ranges up to this size may use value offsets (no keymap) ...
VALUE_OFFSET_DENSITY = 4          # ... when the range is at most this many times the largest segment cardinality
DEFAULT_NUM_GROUPS_LIMIT = 100_000          # InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT
DEFAULT_MAX_INIT_GROUP_HOLDER_CAPACITY = 10_000  # InstancePlanMakerImplV2 :73
# group trim instance defaults (InstancePlanMakerImplV2.java:76-89; GroupByUtils.DEFAULT_MIN_NUM_GROUPS = 5000)
DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE = -1
DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE = 5000
DEFAULT_GROUPBY_TRIM_THRESHOLD = 1_000_000
MAX_TRIM_THRESHOLD = 1_000_000_000   # GroupByOrderByCombineOperator.MAX_TRIM_THRESHOLD: at or above, no resize at all
# batched IN / NOT_IN leaves cross as their literals (values mode, pg_leaf.num_values) unless PG_IN_VALUES=0 (ids)
_IN_VALUES = os.environ.get("PG_IN_VALUES", "1") != "0"


class UnsupportedQuery(Exception):
    """The query shape is not served by the device path (the caller falls back to the CPU plan)."""


# ------------------------------------------------------------------------------------------ lowering

@dataclass
class LoweredLeaf:
    kind: int
    col_id: int
    exclusive: int = 0
    lo: int = 0
    hi: int = 0
    ids: Optional[np.ndarray] = None   # sorted unique int32
    raw: Optional[dict] = None         # PG_LEAF_RAW_SCAN: dtype + values or bounds


_LITERALS: dict = {}   # (id(values), data type) -> (values, coerced literal array): one coercion per predicate


def _coerced_literals(d, values):
    """The IN-list literals coerced to the dictionary's type once per predicate (not once per segment); None when a
    literal does not convert (the per-value path then decides, as Dictionary.indexOf does)."""
    key = (id(values), d.data_type, d.values.dtype.str)
    hit = _LITERALS.get(key)
    if hit is not None and hit[0] is values:
        return hit[1]
    try:
        lit = np.unique(np.asarray([d._coerce(v) for v in values], dtype=d.values.dtype))  # sorted needles
    except (ValueError, OverflowError):
        lit = None
    if len(_LITERALS) > 256:
        _LITERALS.clear()
    _LITERALS[key] = (values, lit)
    return lit


def dict_id_set(d, values) -> np.ndarray:
    """PredicateUtils.getDictIdSet: sorted unique dictIds of the literals present in the dictionary."""
    if d.data_type in ("INT", "LONG", "FLOAT", "DOUBLE"):
        lit = _coerced_literals(d, values)
        if lit is None:
            return np.asarray(sorted({i for i in (d.index_of(v) for v in values) if i >= 0}), dtype=np.int32)
        pos = np.searchsorted(d.values, lit, side="left")
        ok = pos < len(d.values)
        ok[ok] = d.values[pos[ok]] == lit[ok]
        return np.unique(pos[ok]).astype(np.int32)
    return np.asarray(sorted({i for i in (d.index_of(v) for v in values) if i >= 0}), dtype=np.int32)


_RAW_CAST = {"INT": int, "LONG": int, "FLOAT": lambda v: float(np.float32(float(v))), "DOUBLE": float}


def lower_raw_predicate(pred: Predicate, col: Column, col_id: int) -> LoweredLeaf:
    """Raw-value predicate evaluators of a no-dictionary column (Equals / NotEquals / In / NotIn / Range
    PredicateEvaluatorFactory.newRawValueBasedEvaluator): the literals in the column's stored type; an integer
    range folded to closed bounds (exclusive x -> x + 1 / x - 1), a floating range with its inclusivity."""
    t, dt = pred.type, col.data_type
    cast = _RAW_CAST[dt]
    lw = LoweredLeaf(abi.PG_LEAF_RAW_SCAN, col_id)
    lw.raw = {"dtype": dt}
    if t in ("EQ", "NOT_EQ", "IN", "NOT_IN"):
        try:
            vals = sorted({cast(v) for v in pred.values})
        except ValueError:
            raise UnsupportedQuery(f"literal of the wrong type for raw {dt} column {pred.column}")
        lw.exclusive = 1 if t in ("NOT_EQ", "NOT_IN") else 0
        lw.raw["values"] = vals
        return lw
    if t != "RANGE":
        raise UnsupportedQuery(f"predicate type {t}")
    integer = dt in ("INT", "LONG")
    if integer:  # RangePredicateEvaluatorFactory: Integer / Long bounds, folded here to a closed range
        lo, hi = -(1 << 63), (1 << 63) - 1
        try:
            if pred.lower != UNBOUNDED:
                lo = int(pred.lower) + (0 if pred.lower_inclusive else 1)
            if pred.upper != UNBOUNDED:
                hi = int(pred.upper) - (0 if pred.upper_inclusive else 1)
        except ValueError:
            raise UnsupportedQuery(f"non-integer bound on raw {dt} column {pred.column}")
        lw.raw.update(ilo=lo, ihi=hi)
    else:
        lw.raw.update(dlo=-np.inf if pred.lower == UNBOUNDED else cast(pred.lower),
                      dhi=np.inf if pred.upper == UNBOUNDED else cast(pred.upper),
                      lo_inc=1 if pred.lower == UNBOUNDED or pred.lower_inclusive else 0,
                      hi_inc=1 if pred.upper == UNBOUNDED or pred.upper_inclusive else 0)
    return lw


def lower_predicate(pred: Predicate, col: Column, col_id: int, in_ids: Optional[np.ndarray] = None) -> LoweredLeaf:
    """Dictionary-based predicate evaluator + leaf operator choice for one segment's column.  in_ids: the IN / NOT_IN
    literals' dictIds in this segment when already looked up for every segment at once (GpuEngine's pg_dict_id_sets)."""
    if pred.type in ("IS_NULL", "IS_NOT_NULL"):
        # FilterPlanNode.constructPhysicalOperator (plan/FilterPlanNode.java:285-298): without a null value vector
        # (segments built with null handling off, SegmentColumnarIndexCreator.java:291-294) IS NULL is an
        # EmptyFilterOperator and IS NOT NULL a MatchAllFilterOperator
        if getattr(col, "null_vector", None) is not None:
            raise UnsupportedQuery(f"{pred.type} on {pred.column}: null value vectors are not resident")
        return LoweredLeaf(abi.PG_LEAF_EMPTY if pred.type == "IS_NULL" else abi.PG_LEAF_MATCH_ALL, col_id)
    if col.dictionary is None:
        lw = lower_raw_predicate(pred, col, col_id)
        if pred.type == "RANGE" and col.range_index is not None:
            lw.kind = abi.PG_LEAF_RANGE_INDEX   # FilterOperatorUtils.java:60-66: RANGE + range index
        return lw
    d = col.dictionary
    card = len(d)
    excl = 0
    ids = None
    lo = hi = 0
    always_true = always_false = False
    t = pred.type
    if t in ("EQ", "NOT_EQ"):
        i = d.index_of(pred.values[0])
        if t == "EQ":
            if i >= 0:
                ids = np.array([i], dtype=np.int32)
                always_true = card == 1
            else:
                always_false = True
        else:
            excl = 1
            if i >= 0:
                ids = np.array([i], dtype=np.int32)
                always_false = card == 1
            else:
                always_true = True
    elif t in ("IN", "NOT_IN"):
        ids = dict_id_set(d, pred.values) if in_ids is None else in_ids   # PredicateUtils.getDictIdSet
        s = ids
        if t == "IN":
            always_false = len(s) == 0
            always_true = len(s) == card
        else:
            excl = 1
            always_true = len(s) == 0
            always_false = len(s) == card
    elif t == "RANGE":
        # SortedDictionaryBasedRangePredicateEvaluator (RangePredicateEvaluatorFactory.java:115-166)
        if pred.lower == UNBOUNDED:
            start = 0
        else:
            ii = d.insertion_index_of(pred.lower)
            start = -(ii + 1) if ii < 0 else (ii if pred.lower_inclusive else ii + 1)
        if pred.upper == UNBOUNDED:
            end = card
        else:
            ii = d.insertion_index_of(pred.upper)
            end = -(ii + 1) if ii < 0 else (ii + 1 if pred.upper_inclusive else ii)
        lo, hi = start, end
        if end - start <= 0:
            always_false = True
        elif end - start == card:
            always_true = True
    else:
        raise UnsupportedQuery(f"predicate type {t}")
    if always_false:
        return LoweredLeaf(abi.PG_LEAF_EMPTY, col_id)
    if always_true:
        return LoweredLeaf(abi.PG_LEAF_MATCH_ALL, col_id)
    if col.single_value and col.is_sorted:
        kind = abi.PG_LEAF_SORTED
    elif t == "RANGE" and col.range_index is not None:
        kind = abi.PG_LEAF_RANGE_INDEX         # RangeIndexBasedFilterOperator
    elif col.inverted is not None and t != "RANGE":
        kind = abi.PG_LEAF_INVERTED
    else:
        kind = abi.PG_LEAF_SV_SCAN if col.single_value else abi.PG_LEAF_MV_SCAN
    return LoweredLeaf(kind, col_id, excl, lo, hi, ids)


def derived_dictionary(col: Column) -> Dictionary:
    """A raw STRING / BYTES column's derived dictionary: its sorted distinct values (BYTES as lowercase hex), the
    order KeySpace.build's per-doc ids and the resident derived forward index (GpuEngine._upload_derived) number them
    in.  Built once per column."""
    d = getattr(col, "_derived_dict", None)
    if d is None:
        d = Dictionary(col.data_type, np.unique(np.asarray(col.raw_values, dtype=str)).tolist())
        col._derived_dict = d
    return d


def lower_derived_predicate(pred: Predicate, col: Column, col_id: int) -> LoweredLeaf:
    """A predicate on a raw (no-dictionary) STRING / BYTES column.  The reference evaluates it per doc with a raw-value
    evaluator (Equals / NotEquals / In / NotIn / RangePredicateEvaluatorFactory.newRawValueBasedEvaluator: String.equals
    / compareTo, ByteArray equality / ByteArray.compare -- RangePredicateEvaluatorFactory.java:526-580) inside a
    ScanBasedFilterOperator.  Restated over the segment's derived dictionary (sorted distinct values, derived_dictionary):
    a doc matches iff its value's rank is in the dictId set / range the dictionary evaluator computes for the same
    literals.  A raw evaluator is never always-true or always-false (FilterPlanNode only short-cuts those), so the leaf
    stays a scan of every doc: an empty set is the empty range [0, 0), an all-values set its exclusive form.  String
    order is Python's code-point order (Java's compareTo orders UTF-16 units: they differ only beyond U+FFFF)."""
    if pred.type in ("IS_NULL", "IS_NOT_NULL"):
        return lower_predicate(pred, col, col_id)
    d = derived_dictionary(col)
    stand_in = Column(col.name, col.data_type, True, d, col.num_docs, 0, False, col.num_docs)
    lw = lower_predicate(pred, stand_in, col_id)
    if lw.kind == abi.PG_LEAF_EMPTY:
        return LoweredLeaf(abi.PG_LEAF_SV_SCAN, col_id, 0, 0, 0, None)
    if lw.kind == abi.PG_LEAF_MATCH_ALL:
        return LoweredLeaf(abi.PG_LEAF_SV_SCAN, col_id, 1, 0, 0, None)
    return lw


def sum_bound(table: "Table", e: Expr) -> Tuple[int, int, bool]:
    """(pg_agg.sum_exp, pg_agg.sum_exp_lo, PG_SUM_NONFINITE) of a SUM / AVG input: 2^lo <= |x| <= 2^hi for every nonzero
    finite value x of the expression over the table (a*b: the products of the operand bounds; a+b / a-b: the larger
    bound doubled, and a nonzero result is a multiple of the smaller operand's last mantissa bit, 2^-52 of its lower
    bound; an overflow to inf bounds it by DBL_MAX, an underflow by the smallest subnormal), so every GPU that merges
    the plan's partial states cuts the sums into the same exponent windows (pg_internal.h fx_split), and whether some
    input may be +-inf / NaN.  Sent with PG_SUM_BOUNDS, so an all-zero column (0, 0) is unambiguous."""
    hi = [table.abs_bound(c) for c in e.cols]
    lo = [table.abs_low(c) for c in e.cols]
    nonfinite = any(table.has_nonfinite(c) for c in e.cols)
    tiny = 5e-324
    lmin = lambda x, y: y if x == 0 else (x if y == 0 else min(x, y))  # noqa: E731
    if e.op == "COL":
        v, low = hi[0], lo[0]
    elif e.op == "MUL":
        v, low = hi[0] * hi[1], lo[0] * lo[1]
        if lo[0] > 0 and lo[1] > 0 and low == 0:
            low = tiny
    else:
        v, low = hi[0] + hi[1], math.ldexp(lmin(lo[0], lo[1]), -52)
        if lmin(lo[0], lo[1]) > 0 and low == 0:
            low = tiny
    if not math.isfinite(v):
        v, nonfinite = float(np.finfo(np.float64).max), True
    khi = math.frexp(v)[1] if v > 0 else 0            # v < 2^khi
    klo = math.frexp(low)[1] - 1 if low > 0 else khi  # low >= 2^klo
    return khi, klo, nonfinite


def filter_program(f: Optional[FilterContext]) -> Tuple[List[int], List[Predicate]]:
    """Postfix program over leaves (FilterPlanNode.constructPhysicalOperator's tree, in postfix)."""
    ops: List[int] = []
    leaves: List[Predicate] = []

    def walk(n: FilterContext):
        if n.type == "PREDICATE":
            ops.append(len(leaves))
            leaves.append(n.predicate)
        elif n.type == "NOT":
            walk(n.children[0])
            ops.append(abi.PG_OP_NOT)
        else:
            for c in n.children:
                walk(c)
            ops.append(abi.PG_OP_AND(len(n.children)) if n.type == "AND" else abi.PG_OP_OR(len(n.children)))

    if f is not None:
        walk(f)
    return ops, leaves


# ------------------------------------------------------------------------------------------ table

class Table:
    """A set of immutable segments of one table + the table-global key spaces of its columns."""

    def __init__(self, name: str, segments: Sequence[ImmutableSegment]):
        self.name = name
        self.segments = list(segments)
        cols = []
        for s in self.segments:
            for c in s.columns:
                if c not in cols:
                    cols.append(c)
        self.column_ids = {c: i for i, c in enumerate(cols)}
        self._key_spaces: Dict[Tuple[str, bool], "KeySpace"] = {}
        self._abs_bounds: Dict[str, Tuple[float, float, bool]] = {}
        self._searches: dict = {}      # DictSearch per (column, segment list)

    def has_nonfinite(self, column: str) -> bool:
        return self._bounds(column)[2]

    def abs_bound(self, column: str) -> float:
        """The largest |finite value| of a numeric column over every segment of the table (ColumnMetadata min / max:
        the dictionary's ends, or a raw column's values) -- the table-global upper bound of pg_agg.sum_exp."""
        return self._bounds(column)[0]

    def abs_low(self, column: str) -> float:
        """The smallest nonzero |finite value| of a numeric column over the table (0: none) -- the lower bound of
        pg_agg.sum_exp_lo (an integer column: 1)."""
        return self._bounds(column)[1]

    def _bounds(self, column: str) -> Tuple[float, float, bool]:
        hit = self._abs_bounds.get(column)
        if hit is None:
            b, low, nonfinite = 0.0, 0.0, False
            for seg in self.segments:
                c = seg.columns.get(column)
                if c is None:
                    continue
                v = np.asarray(c.raw_values if c.dictionary is None else c.dictionary.values)
                if not v.size or v.dtype.kind not in "iuf":
                    continue
                if v.dtype.kind in "iu":  # integers: the ends bound |v| (a sorted dictionary's ends), nonzero |v| >= 1
                    ends = (v[[0, -1]] if c.dictionary is not None else np.array([v.min(), v.max()])).astype(np.float64)
                    m = float(np.abs(ends).max())
                    b = max(b, m)
                    if m > 0:
                        low = 1.0 if low == 0 else min(low, 1.0)
                    continue
                if c.dictionary is not None and np.isfinite(v[[0, -1]]).all():
                    # a sorted finite dictionary: its ends bound |v|, the smallest nonzero |v| sits around 0
                    b = max(b, float(np.abs(v[[0, -1]]).max()))
                    i = int(np.searchsorted(v, 0.0, side="left"))
                    j = int(np.searchsorted(v, 0.0, side="right"))
                    cand = [abs(float(v[i - 1]))] if i > 0 else []
                    cand += [abs(float(v[j]))] if j < v.size else []
                    if cand:
                        m = min(cand)
                        low = m if low == 0 else min(low, m)
                    continue
                a = np.abs(v.astype(np.float64))
                fin = np.isfinite(a)
                nonfinite |= not bool(fin.all())
                a = a[fin]
                if a.size:
                    b = max(b, float(a.max()))
                    nz = a[a > 0]
                    if nz.size:
                        m = float(nz.min())
                        low = m if low == 0 else min(low, m)
            hit = self._abs_bounds[column] = (b, low, nonfinite)
        return hit

    def data_type(self, column: str) -> str:
        return self.segments[0].columns[column].data_type

    def multi_value(self, column: str) -> bool:
        return any(not s.columns[column].single_value for s in self.segments if column in s.columns)

    def key_space(self, column: str, derive: bool = False) -> "KeySpace":
        ks = self._key_spaces.get((column, derive))
        if ks is None:
            ks = KeySpace.build(column, [s.columns[column] for s in self.segments], derive)
            self._key_spaces[(column, derive)] = ks
        return ks

    def value_space(self, column: str) -> "KeySpace":
        """DISTINCTCOUNT's value ids: the key space, but a raw integer range too wide for a dense value bitmap takes
        the derived dictionary encoding (distinct values only)."""
        ks = self.key_space(column)
        if ks.kind == abi.PG_KEY_VALUE_OFFSET and ks.cardinality > MAX_VALUE_OFFSET_KEYS:
            ks = self.key_space(column, derive=True)
        return ks


def order_keys(values: np.ndarray) -> np.ndarray:
    """Order-preserving int64 images of numeric values in the reference's key order: integers as themselves, FLOAT /
    DOUBLE by Double.compare (-0.0 < 0.0, one NaN above +inf: Double.doubleToLongBits equality, as fastutil's
    Double2IntOpenHashMap keys them in the no-dictionary group-key generators)."""
    v = np.asarray(values)
    if v.dtype.kind in "iu":
        return v.astype(np.int64)
    d = v.astype(np.float64)
    b = d.view(np.int64).copy()
    b[np.isnan(d)] = 0x7FF8000000000000
    return np.where(b >= 0, b, b ^ 0x7FFFFFFFFFFFFFFF)


def order_key_values(keys: np.ndarray, data_type: str) -> list:
    """order_keys' inverse: the values (Python ints / floats) of sorted int64 images."""
    k = np.asarray(keys, dtype=np.int64)
    if data_type in ("INT", "LONG"):
        return k.tolist()
    b = np.where(k >= 0, k, k ^ 0x7FFFFFFFFFFFFFFF)
    d = b.view(np.float64)
    return (d.astype(np.float32).astype(np.float64) if data_type == "FLOAT" else d).tolist()


@dataclass
class KeySpace:
    """Table-global ids for the values of one column (group keys / DISTINCTCOUNT values)."""
    column: str
    kind: int                        # PG_KEY_VALUE_OFFSET or PG_KEY_KEYMAP
    cardinality: int
    base: int = 0
    values: Optional[list] = None    # KEYMAP: global id -> value (sorted union)
    keymaps: Optional[List[np.ndarray]] = None  # per segment dictId -> global id
    _values_np: Optional[np.ndarray] = None
    # raw columns keyed through a host-built dictionary encoding (PG_COL_DERIVED): per segment None (a dictionary
    # segment) or (sorted distinct order keys int64 = the derived dictionary, per-doc ids into it int32)
    derived: Optional[List[Optional[Tuple[np.ndarray, np.ndarray]]]] = None

    @staticmethod
    def build(column: str, cols: List[Column], derive: bool = False) -> "KeySpace":
        """derive: a raw INT / LONG column takes the derived encoding even when its range fits value offsets."""
        dt = cols[0].data_type
        if any(c.dictionary is None for c in cols) and dt in ("STRING", "BYTES"):
            # raw STRING / BYTES (var-byte chunks): every raw segment's values dictionary-encoded on the host (sorted
            # distinct values + per-doc ids), keymapped to the table's sorted union; the derived dictionary holds the
            # values' ranks in that union (the device only needs the keymap), ids = value order (Python str order:
            # code points -- Java's String.compareTo orders UTF-16 code units, which differs only beyond U+FFFF; BYTES
            # as lowercase hex: the unsigned byte order ByteArray.compare uses)
            segu, locs = [], []
            for c in cols:
                if c.dictionary is None:
                    u, local = np.unique(np.asarray(c.raw_values, dtype=str), return_inverse=True)
                    segu.append(u)
                    locs.append(local.astype(np.int32))
                else:
                    segu.append(np.asarray(c.dictionary.values, dtype=str))
                    locs.append(None)
            allu = np.unique(np.concatenate(segu)) if segu else np.zeros(0, dtype=str)
            keymaps = [np.searchsorted(allu, u).astype(np.int32) for u in segu]
            derived = [None if loc is None else (km.astype(np.int64), loc) for km, loc in zip(keymaps, locs)]
            return KeySpace(column, abi.PG_KEY_KEYMAP, len(allu), 0, allu.tolist(), keymaps, derived=derived)
        if any(c.dictionary is None for c in cols):
            if dt not in ("INT", "LONG", "FLOAT", "DOUBLE"):
                raise UnsupportedQuery(f"{column}: raw {dt} column as a key / DISTINCTCOUNT value")
            vals = [c.raw_values if c.dictionary is None else np.asarray(c.dictionary.values) for c in cols]
            if dt in ("INT", "LONG"):
                nz = [v for v in vals if v.size]
                lo = min((int(v.min()) for v in nz), default=0)
                hi = max((int(v.max()) for v in nz), default=0)
                span = hi - lo + 1
                # raw INT / LONG columns: value offsets as 32-bit key ids (pg_key.cardinality), read from the raw
                # values on the device; a group key may span up to 2^32 - 1 values (the device state then hashes
                # them); a DISTINCTCOUNT value set also needs a dense bitmap (checked at its use)
                if span < 1 << 32 and not derive:
                    return KeySpace(column, abi.PG_KEY_VALUE_OFFSET, span, lo)
            # raw FLOAT / DOUBLE, or a wider LONG range: every segment's values dictionary-encoded on the host (sorted
            # distinct values in the reference's key order + per-doc ids), keymapped to the table's sorted union; the
            # device groups on that derived encoding (PG_COL_DERIVED), so segments and GPUs merge by value
            segk, derived = [], []
            for c, v in zip(cols, vals):
                ok = order_keys(v)
                if c.dictionary is None:
                    u, local = np.unique(ok, return_inverse=True)
                    segk.append(u)
                    derived.append((u, local.astype(np.int32)))
                else:
                    segk.append(ok)
                    derived.append(None)
            allk = np.unique(np.concatenate(segk)) if segk else np.zeros(0, dtype=np.int64)
            if len(allk) >= 1 << 31:
                raise UnsupportedQuery(f"{column}: {len(allk)} distinct raw values")
            keymaps = [np.searchsorted(allk, k).astype(np.int32) for k in segk]
            return KeySpace(column, abi.PG_KEY_KEYMAP, len(allk), 0, order_key_values(allk, dt), keymaps,
                            derived=derived)
        if dt in ("INT", "LONG"):
            lo = min(int(c.dictionary.values[0]) for c in cols)
            hi = max(int(c.dictionary.values[-1]) for c in cols)
            span = hi - lo + 1
            # dense enough for direct ids: a sparse range (few values spread wide) would make every group-by state,
            # DISTINCTCOUNT bitmap and merge scale with the range instead of the values
            if span <= MAX_VALUE_OFFSET_KEYS and span <= max(1 << 16, VALUE_OFFSET_DENSITY *
                                                             max(len(c.dictionary) for c in cols)):
                return KeySpace(column, abi.PG_KEY_VALUE_OFFSET, span, lo)
        if dt in ("INT", "LONG", "FLOAT", "DOUBLE"):
            allv = np.unique(np.concatenate([np.asarray(c.dictionary.values) for c in cols]))
            keymaps = [np.searchsorted(allv, np.asarray(c.dictionary.values)).astype(np.int32) for c in cols]
            return KeySpace(column, abi.PG_KEY_KEYMAP, len(allv), 0, list(allv.tolist()), keymaps)
        allv = sorted(set(itertools.chain.from_iterable(c.dictionary.values for c in cols)))
        index = {v: i for i, v in enumerate(allv)}
        keymaps = [np.asarray([index[v] for v in c.dictionary.values], dtype=np.int32) for c in cols]
        return KeySpace(column, abi.PG_KEY_KEYMAP, len(allv), 0, allv, keymaps)

    def value(self, gid: int):
        if self.kind == abi.PG_KEY_VALUE_OFFSET:
            return int(self.base + gid)
        return self.values[gid]

    def values_of(self, gids: np.ndarray) -> set:
        """The value set of an array of global ids (DISTINCTCOUNT's Set intermediate)."""
        if self.kind == abi.PG_KEY_VALUE_OFFSET:
            return set((np.asarray(gids, dtype=np.int64) + self.base).tolist())
        if self._values_np is None:
            self._values_np = np.asarray(self.values, dtype=object)
        return set(self._values_np[np.asarray(gids, dtype=np.int64)].tolist())


# ------------------------------------------------------------------------------------------ results

@dataclass
class ExecutionStats:
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    num_total_docs: int = 0
    num_segments_processed: int = 0
    num_segments_matched: int = 0


@dataclass
class IntermediateResult:
    """Server-side combined result: aggregation-only -> one row under key (); group-by -> value-keyed rows.

    Per aggregation the intermediate value follows the reference's intermediate types:
    COUNT / COUNTMV int, SUM / MIN / MAX float, AVG (sum, count), DISTINCTCOUNT a set of values or
    (device path) the distinct count as an int."""
    aggregations: List[Aggregation]
    group_by: List[str]
    rows: Dict[tuple, list]
    stats: ExecutionStats = field(default_factory=ExecutionStats)
    # IntermediateResultsBlock.isNumGroupsLimitReached: a segment reached the instance's numGroupsLimit
    groups_limit_reached: bool = False
    # the server's combine would have resized its IndexedTable mid-merge (groupTrimThreshold; numResizes > 0)
    trim_threshold_reached: bool = False
    num_groups_merged: Optional[int] = None   # groups of the combined table before the ORDER BY / limit trim


def merge_intermediate(aggs: List[Aggregation], a: list, b: list) -> list:
    """AggregationFunction.merge for each function (e.g. SumAggregationFunction.java:268-278)."""
    out = []
    for ag, x, y in zip(aggs, a, b):
        f = ag.function
        if f in ("COUNT", "COUNTMV", "SUM"):
            out.append(x + y)
        elif f == "MIN":
            out.append(min(x, y))
        elif f == "MAX":
            out.append(max(x, y))
        elif f == "AVG":
            out.append((x[0] + y[0], x[1] + y[1]))
        elif f == "DISTINCTCOUNT":
            if isinstance(x, set) and isinstance(y, set):
                out.append(x | y)
            else:
                raise ValueError("cannot merge distinct counts without value sets")
        else:
            raise ValueError(f)
    return out


def default_row(aggs: List[Aggregation]) -> list:
    """Intermediate values of an aggregation over no docs (each function's initial holder value, e.g.
    MinAggregationFunction DEFAULT_INITIAL_VALUE = +inf, AvgPair(0, 0), an empty DISTINCTCOUNT set)."""
    init = {"COUNT": 0, "COUNTMV": 0, "SUM": 0.0, "MIN": float("inf"), "MAX": float("-inf")}
    return [(0.0, 0) if a.function == "AVG" else set() if a.function == "DISTINCTCOUNT" else init[a.function]
            for a in aggs]


def final_value(ag: Aggregation, v):
    """extractFinalResult of each function (e.g. AvgAggregationFunction.java:276-286)."""
    f = ag.function
    if f in ("COUNT", "COUNTMV"):
        return int(round(v))
    if f in ("SUM", "MIN", "MAX"):
        return float(v)
    if f == "AVG":
        s, c = v
        return float("-inf") if c == 0 else s / c
    if f == "DISTINCTCOUNT":
        return len(v) if isinstance(v, set) else int(v)
    raise ValueError(f)


def reduce_to_rows(query: QueryContext, res: IntermediateResult) -> Tuple[List[str], List[list]]:
    """Broker reduce: final values, ORDER BY (with the remaining select columns as implicit tie-breakers
    only when the ORDER BY names them), LIMIT (BrokerReduceService / GroupByDataTableReducer)."""
    aggs = res.aggregations
    agg_index = {a: i for i, a in enumerate(aggs)}
    names = [s.name() for s in query.select]
    rows_out = []
    if not query.group_by:
        vals = res.rows.get((), None)
        if vals is None:
            vals = default_row(aggs)
        row = []
        for s in query.select:
            row.append(final_value(s.agg, vals[agg_index[s.agg]]))
        return names, [row]
    keyed = []
    for key, vals in res.rows.items():
        finals = [final_value(a, v) for a, v in zip(aggs, vals)]
        keyed.append((key, finals))

    def sort_key(item):
        key, finals = item
        parts = []
        for o in query.order_by:
            if o.kind == "AGG":
                v = finals[agg_index[o.agg]]
            else:
                v = key[query.group_by.index(o.column)]
            parts.append(_Ord(v, o.asc))
        return parts

    if query.order_by:
        keyed.sort(key=sort_key)
    if query.having is not None:
        # GroupByDataTableReducer.reduceToResultTable (:148-165): the broker's table keeps getTableCapacity(limit)
        # records (resultSize = trimSize under HAVING, :232-237); its sorted records are taken in order while fewer
        # than LIMIT rows passed HAVING (HavingFilterHandler.isMatch over the final values)
        keyed = [kf for kf in keyed[:table_capacity(query.limit, 5000)]  # getTableCapacity(limit), GroupByUtils:31
                 if having_match(query.having, query, agg_index, kf[0], kf[1])]
    for key, finals in keyed[:query.limit]:
        row = []
        for s in query.select:
            row.append(key[query.group_by.index(s.column)] if s.kind == "COL" else finals[agg_index[s.agg]])
        rows_out.append(row)
    return names, rows_out


def having_value(e, query: QueryContext, agg_index: dict, key: tuple, finals: list):
    """A HAVING operand's value (PostAggregationHandler.getValueExtractor): an aggregation's final result, a group
    key, a literal; + - * / of them in double arithmetic (the arithmetic transform functions)."""
    if e.kind == "AGG":
        return finals[agg_index[e.agg]]
    if e.kind == "COL":
        return key[query.group_by.index(e.column)]
    if e.kind == "LIT":
        if e.op == "STR":
            return e.value
        return float(e.value) if any(c in e.value for c in ".eE") else int(e.value)
    a, b = (float(having_value(x, query, agg_index, key, finals)) for x in e.args)
    if e.op == "+":
        return a + b
    if e.op == "-":
        return a - b
    if e.op == "*":
        return a * b
    return a / b if b != 0 else (math.copysign(math.inf, a) if a != 0 else math.nan)


def _having_cmp(v, lit: str):
    """(value, literal) in one comparable type: strings compare as strings; an integer value against an integral
    literal exactly; otherwise as doubles (the predicate evaluator of the value column's data type)."""
    if isinstance(v, str):
        return v, lit
    if isinstance(v, int) and not any(c in lit for c in ".eE"):
        return v, int(lit)
    return float(v), float(lit)


def having_match(h, query: QueryContext, agg_index: dict, key: tuple, finals: list) -> bool:
    """HavingFilterHandler.isMatch (query/reduce/HavingFilterHandler.java): AND / OR / NOT of the predicates on the
    row's post-aggregation values (no null handling: IS NULL never matches)."""
    if h.type == "AND":
        return all(having_match(c, query, agg_index, key, finals) for c in h.children)
    if h.type == "OR":
        return any(having_match(c, query, agg_index, key, finals) for c in h.children)
    if h.type == "NOT":
        return not having_match(h.children[0], query, agg_index, key, finals)
    p = h.predicate
    v = having_value(h.lhs, query, agg_index, key, finals)
    if p.type in ("IS_NULL", "IS_NOT_NULL"):
        return p.type == "IS_NOT_NULL"
    if isinstance(v, float) and math.isnan(v):
        return p.type in ("NOT_EQ", "NOT_IN")
    if p.type in ("EQ", "IN", "NOT_EQ", "NOT_IN"):
        hit = any(a == b for a, b in (_having_cmp(v, x) for x in p.values))
        return hit if p.type in ("EQ", "IN") else not hit
    ok = True
    if p.lower != UNBOUNDED:
        a, b = _having_cmp(v, p.lower)
        ok &= a >= b if p.lower_inclusive else a > b
    if p.upper != UNBOUNDED:
        a, b = _having_cmp(v, p.upper)
        ok &= a <= b if p.upper_inclusive else a < b
    return ok


# ------------------------------------------------------------------------------------------ group trim

@dataclass
class InstanceConfig:
    """The pinot.server.query.executor.* settings InstancePlanMakerImplV2 reads (plan/maker/
    InstancePlanMakerImplV2.java:67-89 keys, :132-150 the QueryExecutorConfig constructor): num.groups.limit,
    max.init.group.holder.capacity, min.segment / min.server group trim sizes, groupby.trim.threshold.

    numGroupsLimit is an INSTANCE setting only: applyQueryOptions (:223) sets queryContext.setNumGroupsLimit from it, and
    QueryOptionsUtils has no such query option -- an OPTION(numGroupsLimit=...) in the SQL changes nothing (as in
    Pinot 0.11).  The constructor's preconditions hold here too (:138-140, :144-145)."""
    num_groups_limit: int = DEFAULT_NUM_GROUPS_LIMIT
    min_segment_group_trim_size: int = DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE
    min_server_group_trim_size: int = DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE
    groupby_trim_threshold: int = DEFAULT_GROUPBY_TRIM_THRESHOLD
    max_init_group_holder_capacity: int = DEFAULT_MAX_INIT_GROUP_HOLDER_CAPACITY

    def __post_init__(self):
        if self.max_init_group_holder_capacity > self.num_groups_limit:
            raise ValueError(f"Invalid configuration: maxInitialResultHolderCapacity: "
                             f"{self.max_init_group_holder_capacity} must be smaller or equal to numGroupsLimit: "
                             f"{self.num_groups_limit}")
        if self.groupby_trim_threshold <= 0:
            raise ValueError(f"Invalid configurable: groupByTrimThreshold: {self.groupby_trim_threshold} must be "
                             f"positive")

    @staticmethod
    def with_groups_limit(limit: int, **kw) -> "InstanceConfig":
        """An instance whose num.groups.limit is `limit` (and max.init.group.holder.capacity lowered to it when it is
        below the 10 000 default, as the precondition requires)."""
        return InstanceConfig(num_groups_limit=limit,
                              max_init_group_holder_capacity=min(DEFAULT_MAX_INIT_GROUP_HOLDER_CAPACITY, limit), **kw)


@dataclass(frozen=True)
class GroupTrim:
    """What a server keeps of a group-by result.  segment_size: per-segment trim capacity (None = off); server_size:
    rows of the server's combined result (None = every group); ordered: the kept rows are the top of the ORDER BY
    (else `server_size` arbitrary groups -- here the smallest key ids); threshold: IndexedTable's trimThreshold."""
    segment_size: Optional[int]
    server_size: Optional[int]
    ordered: bool
    threshold: int


def table_capacity(limit: int, min_num_groups: int) -> int:
    """GroupByUtils.getTableCapacity (util/GroupByUtils.java:40-42): max(limit * 5, minNumGroups)."""
    return max(limit * 5, min_num_groups)


def _int_option(query: QueryContext, name: str) -> Optional[int]:
    v = query.options.get(name)
    return None if v is None else int(v)


def group_trim(query: QueryContext, config: Optional[InstanceConfig] = None) -> GroupTrim:
    """InstancePlanMakerImplV2.applyQueryOptions (:189-240: the minSegmentGroupTrimSize / minServerGroupTrimSize query
    options override the instance config; groupTrimThreshold is instance-level) followed by the trims those settings
    drive: AggregationGroupByOrderByOperator.getNextBlock (operator/query/AggregationGroupByOrderByOperator.java:
    118-132: a segment with ORDER BY and more groups than getTableCapacity(limit, minSegmentGroupTrimSize) keeps that
    many) and the GroupByOrderByCombineOperator constructor (operator/combine/GroupByOrderByCombineOperator.java:79-93:
    ORDER BY -> getTableCapacity(limit, minServerGroupTrimSize), none -> limit, minServerGroupTrimSize <= 0 -> every
    group), whose IndexedTable.finish keeps that many (data/table/IndexedTable.java:147-158)."""
    cfg = config or InstanceConfig()
    seg_min = _int_option(query, "minSegmentGroupTrimSize")
    seg_min = cfg.min_segment_group_trim_size if seg_min is None else seg_min
    srv_min = _int_option(query, "minServerGroupTrimSize")
    srv_min = cfg.min_server_group_trim_size if srv_min is None else srv_min
    ordered = bool(query.order_by)
    seg = table_capacity(query.limit, seg_min) if ordered and seg_min > 0 else None
    if srv_min > 0:
        # ORDER BY or HAVING -> getTableCapacity(limit, minServerGroupTrimSize) (:82-84); neither -> LIMIT
        srv = table_capacity(query.limit, srv_min) if ordered or query.having is not None else query.limit
        threshold = cfg.groupby_trim_threshold
    else:
        srv, threshold = None, (1 << 31) - 1
    return GroupTrim(seg, srv, ordered, threshold)


def order_values(query: QueryContext, aggs: List[Aggregation], key: tuple, row: list) -> list:
    """TableResizer's OrderByValueExtractors (data/table/TableResizer.java:121-150): a group-by expression's value or
    the aggregation's final result (AggregationFunctionExtractor -> extractFinalResult)."""
    out = []
    for o in query.order_by:
        if o.kind == "AGG":
            i = aggs.index(o.agg)
            out.append(final_value(aggs[i], row[i]))
        else:
            out.append(key[query.group_by.index(o.column)])
    return out


def top_groups(query: QueryContext, aggs: List[Aggregation], rows: Dict[tuple, list], size: int) -> Dict[tuple, list]:
    """TableResizer.getTopRecords(recordsMap, size) (TableResizer.java:248-310) over value-keyed rows: the `size`
    groups first under the ORDER BY; groups the ORDER BY ties at the boundary are taken in ascending key order (the
    reference's heap leaves that choice arbitrary).  Without an ORDER BY: the `size` smallest keys (an IndexedTable
    without ORDER BY keeps the first `size` keys it sees, IndexedTable.java:95-103)."""
    if len(rows) <= size:
        return rows
    if query.order_by:
        items = sorted(rows.items(), key=lambda kv: kv[0])
        items.sort(key=lambda kv: [_Ord(v, o.asc) for v, o in zip(order_values(query, aggs, kv[0], kv[1]),
                                                                   query.order_by)])
    else:
        items = sorted(rows.items(), key=lambda kv: kv[0])
    return dict(items[:size])


# ------------------------------------------------------------------------------------------ filtered aggregations

def has_filtered_aggregations(query: QueryContext) -> bool:
    """QueryContext.isHasFilteredAggregations (QueryContext.java:261, set at :531-533)."""
    return any(a.filter is not None for a in query.aggregations)


def filtered_aggregation_passes(query: QueryContext) -> List[Tuple[QueryContext, List[int]]]:
    """AggregationPlanNode.buildFilteredAggOperator (plan/AggregationPlanNode.java:87-146): one pass per distinct
    aggregation filter f, over CombinedFilterOperator(main, f) = main AND f (CombinedFilterOperator.java:56-61), plus
    the main filter's pass for the non-filtered aggregations (always run, even with none: its docs count in the
    statistics).  Returns [(pass query, indices into query.aggregations)], the main pass last.  A pass with no
    aggregation of its own carries COUNT(*) so that the engines report its docs."""
    aggs = query.aggregations
    groups: Dict[str, Tuple[FilterContext, List[int]]] = {}
    plain: List[int] = []
    for i, a in enumerate(aggs):
        if a.filter is None:
            plain.append(i)
            continue
        groups.setdefault(filter_str(a.filter), (a.filter, []))[1].append(i)
    out = []
    for f, idx in groups.values():
        combined = f if query.filter is None else FilterContext(
            "AND", (query.filter.children if query.filter.type == "AND" else [query.filter]) +
            (f.children if f.type == "AND" else [f]))
        out.append((_pass_query(query, combined, [Aggregation(aggs[i].function, aggs[i].arg, mv=aggs[i].mv) for i in idx]), idx))
    out.append((_pass_query(query, query.filter, [aggs[i] for i in plain] or [Aggregation("COUNT", Expr("STAR"))]),
                plain))
    return out


def _pass_query(query: QueryContext, filt, aggs: List[Aggregation]) -> QueryContext:
    return QueryContext(query.table, [SelectItem("AGG", agg=a) for a in aggs], filt, [], [], query.limit,
                        dict(query.options))


def assemble_filtered(query: QueryContext, passes, results: List["IntermediateResult"]) -> "IntermediateResult":
    """FilteredAggregationOperator.getNextBlock (operator/query/FilteredAggregationOperator.java:70-98): each
    function's result from its pass; numDocsScanned and numEntriesScannedInFilter summed over the passes,
    numEntriesScannedPostFilter = sum of (pass docs x the columns of ALL the aggregations) -- every pass projects
    the whole aggregation expression set (buildTransformOperatorForFilteredAggregates, :159-166); numTotalDocs and
    the segment counts from the main pass (its docs contain every other pass's).

    The reference's buildFilterOperatorInternal (AggregationPlanNode.java:110-135) tests `inputPair.getLeft() != null`
    (the function, never null) where the filter is meant, so the non-filtered functions run as one more
    CombinedFilterOperator(main, match-all) pass and the main pass itself runs with no function: with any non-filtered
    function the main pass's docs count twice (InnerSegmentAggregationSingleValueQueriesTest.java:73-103 expects
    180 000 docs for 5 functions over 30 000).  Both passes select the same docs, so the main pass runs once here and its
    statistics are added a second time."""
    aggs = query.aggregations
    row = [None] * len(aggs)
    st = ExecutionStats()
    projected = len({c for a in aggs if a.function != "COUNT" for c in a.arg.cols})
    for n, ((pq, idx), res) in enumerate(zip(passes, results)):
        vals = res.rows.get((), None) or default_row(pq.aggregations)
        for k, i in enumerate(idx):
            row[i] = vals[k]
        times = 2 if n == len(passes) - 1 and idx else 1
        st.num_docs_scanned += times * res.stats.num_docs_scanned
        st.num_entries_scanned_in_filter += times * res.stats.num_entries_scanned_in_filter
        st.num_entries_scanned_post_filter += times * res.stats.num_docs_scanned * projected
    main = results[-1].stats
    st.num_total_docs = main.num_total_docs
    st.num_segments_processed = main.num_segments_processed
    st.num_segments_matched = main.num_segments_matched
    return IntermediateResult(aggs, [], {(): row}, st)


def execute_filtered(run, query: QueryContext) -> "IntermediateResult":
    """Runs the passes of a query with filtered aggregations through `run(pass_query) -> IntermediateResult`."""
    passes = filtered_aggregation_passes(query)
    return assemble_filtered(query, passes, [run(pq) for pq, _ in passes])


class _Ord:
    __slots__ = ("v", "asc")

    def __init__(self, v, asc):
        self.v = v
        self.asc = asc

    def __lt__(self, other):
        return self.v < other.v if self.asc else self.v > other.v

    def __eq__(self, other):
        return self.v == other.v


# ------------------------------------------------------------------------------------------ C plan

# ------------------------------------------------------------------------------------------ query shape

def _filter_shape(f: Optional[FilterContext]):
    if f is None:
        return None
    if f.type == "PREDICATE":
        p = f.predicate
        return ("P", p.type, p.column, p.lower == UNBOUNDED, p.upper == UNBOUNDED, p.lower_inclusive,
                p.upper_inclusive)
    return (f.type, tuple(_filter_shape(c) for c in f.children))


def query_shape(q: QueryContext) -> tuple:
    """A query with its filter's literals left out: two queries of one shape lower to the same plan but for the
    leaves (CPlan.relower) -- a server's parametrised queries with fresh literals."""
    import dataclasses
    return _filter_shape(q.filter), repr(dataclasses.replace(q, filter=None))


# ------------------------------------------------------------------------------------------ vectorized leaf lowering

def _ctypes_dtype(st) -> np.dtype:
    """A numpy structured dtype with the exact layout of a ctypes Structure (pointers as uint64)."""
    kinds = {C.c_uint32: "<u4", C.c_int32: "<i4", C.c_int64: "<i8", C.c_uint64: "<u8", C.c_double: "<f8",
             C.c_void_p: "<u8"}
    names, formats, offsets = [], [], []
    for name, ty in st._fields_:
        names.append(name)
        formats.append(kinds.get(ty, "<u8"))   # POINTER(...) fields: 8-byte addresses
        offsets.append(getattr(st, name).offset)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": C.sizeof(st)})


PG_LEAF_DTYPE = _ctypes_dtype(abi.pg_leaf)
_NUMERIC_DICT = ("INT", "LONG", "FLOAT", "DOUBLE")
_SEARCH_MAX_ENTRIES = 8 << 20   # columns whose dictionaries hold more entries over the segments search per segment


class DictSearch:
    """The sorted dictionaries of one numeric column over a list of segments, searchable for every segment at once:
    each value's rank in the union of the dictionaries, offset by segment (a sorted int64 key), so the insertion point
    of a literal in every segment's dictionary is two vectorized searches instead of one binary search per segment
    (BaseImmutableDictionary.binarySearch, once per segment per literal in the reference's predicate evaluators)."""

    def __init__(self, dicts):
        vals = [d.values for d in dicts]
        sizes = np.array([len(v) for v in vals], dtype=np.int64)
        self.off = np.concatenate([[0], np.cumsum(sizes)])
        allv = np.concatenate(vals) if len(vals) else np.zeros(0)
        self.union = np.unique(allv)
        span = len(self.union) + 1
        seg = np.repeat(np.arange(len(vals), dtype=np.int64), sizes)
        self.key = seg * span + np.searchsorted(self.union, allv)
        self.base = np.arange(len(vals), dtype=np.int64) * span
        self.allv = allv
        self.sizes = sizes

    def count_below(self, v, inclusive: bool) -> np.ndarray:
        """Per segment: the number of dictionary values < v (or <= v)."""
        r = np.searchsorted(self.union, v, side="right" if inclusive else "left")
        return np.searchsorted(self.key, self.base + r, side="left") - self.off[:-1]

    def index_of(self, v) -> np.ndarray:
        """Per segment: the dictId of v, or -1 (Dictionary.indexOf)."""
        i = self.count_below(v, False)
        at = np.minimum(self.off[:-1] + i, max(len(self.allv) - 1, 0))
        hit = (i < self.sizes) & (self.allv[at] == v) if len(self.allv) else np.zeros(len(i), dtype=bool)
        return np.where(hit, i, -1)


def _dict_search(table: "Table", column: str, segments) -> Optional[DictSearch]:
    key = (column, tuple(id(s) for s in segments))
    cache = table._searches
    hit = cache.get(key)
    if hit is None:
        dicts = [s.columns[column].dictionary for s in segments]
        if sum(len(d) for d in dicts) > _SEARCH_MAX_ENTRIES:
            return None
        hit = cache[key] = (DictSearch(dicts), segments)
    return hit[0]


def lower_leaf_vectorized(table: "Table", pred: Predicate, segments, col_id: int, batch) -> Optional[dict]:
    """lower_predicate for one leaf over every segment at once, as field arrays of the pg_leaf table (None: a shape
    the vectorized form does not cover -- the per-segment path lowers it).  Same semantics: predicate evaluator ->
    dictId range / set per segment, the isAlwaysTrue / isAlwaysFalse shortcuts, the leaf operator choice."""
    cols = [s.columns.get(pred.column) for s in segments]
    if any(c is None or c.dictionary is None for c in cols):
        return None
    d0 = cols[0].dictionary
    if d0.data_type not in _NUMERIC_DICT or any(c.dictionary.data_type != d0.data_type for c in cols):
        return None
    t = pred.type
    if t not in ("RANGE", "EQ", "NOT_EQ", "IN", "NOT_IN"):
        return None
    S = len(segments)
    card = np.array([len(c.dictionary) for c in cols], dtype=np.int64)
    sv = np.array([c.single_value for c in cols], dtype=bool)
    srt = np.array([c.is_sorted for c in cols], dtype=bool)
    rng = np.array([c.range_index is not None for c in cols], dtype=bool)
    inv = np.array([c.inverted is not None for c in cols], dtype=bool)
    out = {"lo": np.zeros(S, np.int64), "hi": np.zeros(S, np.int64), "exclusive": np.zeros(S, np.int64),
           "num_ids": np.zeros(S, np.int64), "ids": np.zeros(S, np.uint64), "values": np.zeros(S, np.uint64),
           "num_values": np.zeros(S, np.int64), "keep": []}
    if t == "RANGE" or t in ("EQ", "NOT_EQ"):
        ds = _dict_search(table, pred.column, segments)
        if ds is None:
            return None
        try:
            if t == "RANGE":
                start = np.zeros(S, np.int64) if pred.lower == UNBOUNDED else \
                    ds.count_below(d0._coerce(pred.lower), not pred.lower_inclusive)
                end = card.copy() if pred.upper == UNBOUNDED else \
                    ds.count_below(d0._coerce(pred.upper), bool(pred.upper_inclusive))
            else:
                idx = ds.index_of(d0._coerce(pred.values[0]))
        except (ValueError, OverflowError):
            return None
        if t == "RANGE":
            out["lo"], out["hi"] = start, end
            always_false = end - start <= 0
            always_true = end - start == card
        else:
            found = idx >= 0
            ids = np.ascontiguousarray(np.where(found, idx, 0), dtype=np.int32)
            out["keep"].append(ids)
            out["ids"] = np.where(found, ids.ctypes.data + 4 * np.arange(S, dtype=np.uint64), 0).astype(np.uint64)
            out["num_ids"] = found.astype(np.int64)
            if t == "EQ":
                always_false, always_true = ~found, found & (card == 1)
            else:
                out["exclusive"][:] = 1
                always_false, always_true = found & (card == 1), ~found
    else:
        if batch is None:
            return None
        ids2, counts, wide = batch
        cnt = counts.astype(np.int64)
        n = ids2.shape[1]
        rows = ids2.ctypes.data + 4 * n * np.arange(S, dtype=np.uint64)
        first = ids2[:, 0].astype(np.int64)
        last = ids2[np.arange(S), np.maximum(cnt - 1, 0)].astype(np.int64)
        has = cnt > 0
        contiguous = last - first + 1 == cnt
        out["num_ids"] = cnt
        out["keep"].append(ids2)
        if t == "IN":
            always_false, always_true = ~has, cnt == card
        else:
            out["exclusive"][:] = 1
            always_false, always_true = has & (cnt == card), ~has
    # leaf operator (FilterOperatorUtils.getLeafFilterOperator): sorted index, range index (RANGE), inverted index
    # (not RANGE), else a scan
    kind = np.where(sv, abi.PG_LEAF_SV_SCAN, abi.PG_LEAF_MV_SCAN)
    if t != "RANGE":
        kind = np.where(inv, abi.PG_LEAF_INVERTED, kind)
    else:
        kind = np.where(rng, abi.PG_LEAF_RANGE_INDEX, kind)
    kind = np.where(sv & srt, abi.PG_LEAF_SORTED, kind)
    kind = np.where(always_true, abi.PG_LEAF_MATCH_ALL, kind)
    kind = np.where(always_false, abi.PG_LEAF_EMPTY, kind)
    out["kind"] = kind
    if t in ("IN", "NOT_IN"):
        shortcut = always_true | always_false
        # values mode: the literals (one array for every segment) cross instead of a non-contiguous dictId list of a
        # scan leaf; the device finds the dictIds in the resident dictionary
        vmode = (~shortcut & has & ~contiguous & ((kind == abi.PG_LEAF_SV_SCAN) | (kind == abi.PG_LEAF_MV_SCAN))
                 if _IN_VALUES else np.zeros(S, bool))
        keep_ids = ~shortcut & has
        out["ids"] = np.where(keep_ids & ~vmode, rows, 0).astype(np.uint64)
        out["values"] = np.where(vmode, wide.ctypes.data, 0).astype(np.uint64)
        out["num_values"] = np.where(vmode, len(wide), 0)
        out["num_ids"] = np.where(keep_ids, cnt, 0)
        out["keep"].append(wide)
    else:
        shortcut = always_true | always_false
        if t != "RANGE":
            out["ids"] = np.where(shortcut, 0, out["ids"]).astype(np.uint64)
            out["num_ids"] = np.where(shortcut, 0, out["num_ids"])
    for f in ("exclusive",):  # the shortcut leaves carry no exclusivity (LoweredLeaf of EMPTY / MATCH_ALL)
        out[f] = np.where(shortcut, 0, out[f])
    out["lo"] = np.where(shortcut, 0, out["lo"])
    out["hi"] = np.where(shortcut, 0, out["hi"])
    return out


class CPlan:
    """Owns every ctypes array a pg_plan points to (kept alive while the plan is in use)."""

    def __init__(self, table: Table, query: QueryContext, segments: Sequence[ImmutableSegment],
                 seg_keys: Sequence[int], flags: int = 0, trim=False, id_sets=None,
                 config: Optional["InstanceConfig"] = None, derived_ids: bool = False):
        """config: the server instance's settings (InstanceConfig; numGroupsLimit, trim sizes, trim threshold).
        flags: PG_PLAN_*.  trim (group-by only): True -- the device applies the query's ORDER BY / LIMIT (boundary
        ties kept: a final, single-server answer); "server" -- the device keeps exactly the rows the reference server's
        combine keeps (group_trim(query, config): getTableCapacity(limit, minServerGroupTrimSize) under the ORDER BY,
        `limit` groups without one, all of them when the server trim is off); an int -- exactly that many under the
        ORDER BY (the per-segment trim).
        id_sets(col_id, data_type, literals, seg_keys) -> (ids [S, n] int32, counts [S]): the IN / NOT_IN literals'
        dictIds in every segment in one call (GpuEngine: pg_dict_id_sets on the resident dictionaries); None = per
        segment on the host.
        derived_ids: key / DISTINCTCOUNT columns whose key space is a host-built dictionary encoding of a raw column
        (KeySpace.derived) are named col_id | PG_COL_DERIVED, the device's resident copy of that encoding (GpuEngine);
        the oracle reads the raw column itself."""
        self.table = table
        self.query = query
        self.config = config or InstanceConfig()
        self.aggs = query.aggregations
        if has_filtered_aggregations(query):
            raise UnsupportedQuery("filtered aggregations run as one plan per filter (execute_filtered)")
        self._keep = []
        self.derived_ids = derived_ids
        cid = table.column_ids
        ops, preds = filter_program(query.filter)
        self.leaf_preds = preds
        L = len(preds)
        S = len(segments)
        seg_arr = self._lower_leaves(table, segments, seg_keys, preds, id_sets)
        ops_arr = (C.c_int32 * max(len(ops), 1))(*ops)
        self._keep.append(ops_arr)

        aggs = (abi.pg_agg * max(len(self.aggs), 1))()
        for i, ag in enumerate(self.aggs):
            aggs[i].fn = abi.AGG_CODES[ag.function]
            e = ag.arg
            if ag.function != "COUNT":
                if e.op == "STAR":
                    raise UnsupportedQuery(f"{ag.function}(*)")
                aggs[i].col_a = cid[e.cols[0]]
                aggs[i].op = {"COL": abi.PG_EXPR_COL, "MUL": abi.PG_EXPR_MUL, "ADD": abi.PG_EXPR_ADD,
                              "SUB": abi.PG_EXPR_SUB}[e.op]
                if e.op != "COL":
                    if ag.function not in ("SUM", "MIN", "MAX", "AVG"):
                        raise UnsupportedQuery(f"{ag.function} over an expression")
                    aggs[i].col_b = cid[e.cols[1]]
                for c in e.cols:
                    if table.data_type(c) in ("STRING", "BYTES") and ag.function not in ("DISTINCTCOUNT", "COUNTMV"):
                        raise UnsupportedQuery(f"{ag.function} on non-numeric column {c}")
                    # the SV functions read getXxxValuesSV / getDictionaryIdsSV and COUNTMV getNumMVEntries: a
                    # function over the other kind of column fails in the reference too (SUMMV, DISTINCTCOUNTMV, ...
                    # are other functions)
                    if table.multi_value(c) != (ag.function == "COUNTMV" or ag.mv):
                        raise UnsupportedQuery(f"{ag.name} over {'multi' if table.multi_value(c) else 'single'}"
                                               f"-value column {c}")
                if ag.mv:
                    if e.op != "COL":
                        raise UnsupportedQuery(f"{ag.name} over an expression")
                    aggs[i].flags = abi.PG_AGG_MV_VALUES
                if ag.function == "DISTINCTCOUNT":
                    ks = table.value_space(e.cols[0])
                    if derived_ids and ks.derived is not None:
                        aggs[i].col_a |= abi.PG_COL_DERIVED
                    aggs[i].key_kind = ks.kind
                    aggs[i].key_cardinality = ks.cardinality
                    aggs[i].key_base = ks.base
                if ag.function in ("SUM", "AVG"):
                    aggs[i].sum_exp, aggs[i].sum_exp_lo, nonfinite = sum_bound(table, e)
                    aggs[i].sum_flags = abi.PG_SUM_BOUNDS | (abi.PG_SUM_NONFINITE if nonfinite else 0)
        self._keep.append(aggs)
        keys = (abi.pg_key * max(len(query.group_by), 1))()
        self.key_spaces = []
        for k, col in enumerate(query.group_by):
            # a raw (no-dictionary) key groups by value (NoDictionarySingleColumnGroupKeyGenerator /
            # NoDictionaryMultiColumnGroupKeyGenerator, DefaultGroupByExecutor.java:85-94): INT / LONG by value offset,
            # FLOAT / DOUBLE / wide LONG through a derived dictionary encoding (KeySpace.build)
            ks = table.key_space(col)
            self.key_spaces.append(ks)
            keys[k].col_id = cid[col] | (abi.PG_COL_DERIVED if derived_ids and ks.derived is not None else 0)
            keys[k].kind = ks.kind
            keys[k].cardinality = ks.cardinality
            keys[k].base = ks.base
        # a multi-value key groups each value of a doc's list (DictionaryBasedGroupKeyGenerator :188-200); several group
        # each tuple of the cartesian product of their lists (getIntRawKeys :472-540)
        self._keep.append(keys)

        p = abi.pg_plan()
        p.abi_version = abi.PG_ABI_VERSION
        p.num_segments = S
        p.segments = seg_arr
        p.num_leaves = L
        p.num_ops = len(ops)
        p.ops = ops_arr
        p.num_aggs = len(self.aggs)
        p.num_keys = len(query.group_by)
        p.aggs = aggs
        p.keys = keys
        # InstancePlanMakerImplV2.applyQueryOptions (:223): the instance's num.groups.limit, never a query option
        p.num_groups_limit = self.config.num_groups_limit
        p.flags = flags
        gt = group_trim(query, self.config) if query.group_by else None
        if gt is not None and gt.ordered and gt.server_size is not None and gt.threshold < MAX_TRIM_THRESHOLD:
            p.trim_threshold = gt.threshold   # flags PG_RESULT_TRIM_THRESHOLD_REACHED when the merge reaches it
        size, exact = query.limit, False
        if query.having is not None and query.order_by:
            # HAVING runs after this cut (reduce_to_rows): keep the broker's table capacity so that groups failing
            # HAVING cannot take LIMIT slots -- GroupByDataTableReducer keeps getTableCapacity(limit) sorted records and
            # walks them until `limit` rows pass HAVING (:148-165)
            size = table_capacity(query.limit, 5000)
        if trim == "server":   # the reference server's IndexedTable result (group_trim); every group when trim is off
            size, exact = group_trim(query, config).server_size, True
        elif not isinstance(trim, bool) and isinstance(trim, int):   # an explicit exact size (per-segment trims)
            size, exact = trim, True
        if trim is not False and query.group_by and size is not None and (exact or query.order_by):
            p.limit = size
            if exact:
                p.flags |= abi.PG_PLAN_EXACT_LIMIT
        if trim is not False and query.group_by and query.order_by and size is not None:
            order = (abi.pg_order * len(query.order_by))()
            for i, o in enumerate(query.order_by):
                if o.kind == "AGG":
                    order[i].kind, order[i].index = abi.PG_ORDER_AGG, self.aggs.index(o.agg)
                elif o.column in query.group_by:
                    order[i].kind, order[i].index = abi.PG_ORDER_KEY, query.group_by.index(o.column)
                else:
                    raise UnsupportedQuery(f"ORDER BY {o.column}")
                order[i].desc = 0 if o.asc else 1
            self._keep.append(order)
            p.num_order = len(query.order_by)
            p.order = order
        self.plan = p
        self.ops = ops
        # the shared image is built once (under the lock: cached plans are shared by threads); every thread gets its own
        # copy, whose header carries that call's scalars
        self._image = None
        self._image_lock = threading.Lock()
        self._tls = threading.local()

    def _lower_leaves(self, table: Table, segments, seg_keys, preds, id_sets):
        """Every segment's leaves (the filter's predicates lowered into dictId space) as one pg_leaf table and the
        pg_segment_ref array pointing into it (CPlan.__init__, and relower for a query of the same shape)."""
        cid = table.column_ids
        S, L = len(segments), len(preds)
        self._leaf_keep = []
        self._lowered = None
        seg_arr = (abi.pg_segment_ref * max(S, 1))()
        batch = self._batched_in_ids(preds, segments, seg_keys, cid, id_sets) if id_sets is not None and S > 1 else {}
        self._leaf_keep.extend(b[2] for b in batch.values())  # the literal arrays values-mode leaves point to
        # the leaves of every segment as ONE table in pg_leaf's layout ([segment][leaf]), each segment's row pointed to
        # by its pg_segment_ref; a leaf is lowered for all segments at once where the vectorized form covers it
        # (lower_leaf_vectorized), else segment by segment (lower_predicate)
        Lc = max(L, 1)
        tab = np.zeros((max(S, 1), Lc), dtype=PG_LEAF_DTYPE)
        self._leaf_tab = tab
        self._vec: Dict[int, dict] = {}
        self._per_seg: Dict[Tuple[int, int], LoweredLeaf] = {}
        self._batch = batch
        for p in preds:
            if p.column not in cid or any(p.column not in seg.columns for seg in segments):
                raise UnsupportedQuery(f"unknown column {p.column}")
        derived_bit = abi.PG_COL_DERIVED if getattr(self, "derived_ids", False) else 0
        for li, p in enumerate(preds):
            b = batch.get(li)
            vec = lower_leaf_vectorized(table, p, segments, cid[p.column], b) if S > 1 else None
            if vec is not None:
                col = tab[:S, li]
                col["col_id"] = cid[p.column]
                for f in ("kind", "exclusive", "lo", "hi", "num_ids", "ids", "values", "num_values"):
                    col[f] = vec[f]
                self._leaf_keep.extend(vec["keep"])
                self._vec[li] = vec
                continue
            for si, seg in enumerate(segments):
                c = seg.columns[p.column]
                if c.dictionary is None and c.data_type in ("STRING", "BYTES"):
                    # the device holds a raw STRING / BYTES column only as its derived encoding (col | DERIVED)
                    lw = lower_derived_predicate(p, c, cid[p.column] | derived_bit)
                else:
                    lw = lower_predicate(p, c, cid[p.column], None if b is None else b[0][si, :b[1][si]])
                self._per_seg[(si, li)] = lw
                r = tab[si, li]
                r["kind"], r["col_id"], r["exclusive"], r["lo"], r["hi"] = lw.kind, lw.col_id, lw.exclusive, lw.lo, lw.hi
                if lw.ids is not None and len(lw.ids):
                    arr = np.ascontiguousarray(lw.ids, dtype=np.int32)
                    r["num_ids"] = len(arr)
                    if b is not None and _IN_VALUES and lw.kind in (abi.PG_LEAF_SV_SCAN, abi.PG_LEAF_MV_SCAN) and \
                            int(arr[-1]) - int(arr[0]) + 1 != len(arr):
                        # values mode: the predicate's literals (one array for every segment); the device finds their
                        # dictIds in the resident dictionary (a contiguous id set still crosses as ids: a RANGE leaf)
                        r["values"] = b[2].ctypes.data
                        r["num_values"] = len(b[2])
                    else:
                        self._leaf_keep.append(arr)
                        r["ids"] = arr.ctypes.data
                if lw.raw is not None:
                    raw = lw.raw
                    if "values" in raw:  # int64 for INT / LONG columns, float64 for FLOAT / DOUBLE
                        arr = np.ascontiguousarray(raw["values"], dtype=np.int64 if raw["dtype"] in ("INT", "LONG")
                                                   else np.float64)
                        self._leaf_keep.append(arr)
                        r["num_ids"] = len(arr)
                        r["values"] = arr.ctypes.data
                    else:
                        r["ilo"], r["ihi"] = raw.get("ilo", 0), raw.get("ihi", 0)
                        r["dlo"], r["dhi"] = raw.get("dlo", 0.0), raw.get("dhi", 0.0)
                        r["lo_inclusive"], r["hi_inclusive"] = raw.get("lo_inc", 1), raw.get("hi_inc", 1)
        base = tab.ctypes.data
        seg_tab = np.frombuffer(seg_arr, dtype=_ctypes_dtype(abi.pg_segment_ref), count=max(S, 1))
        seg_tab["seg_key"][:S] = np.asarray(seg_keys, dtype=np.uint64)
        seg_tab["num_docs"][:S] = [seg.num_docs for seg in segments]
        seg_tab["leaves"][:S] = base + np.arange(S, dtype=np.uint64) * (Lc * PG_LEAF_DTYPE.itemsize)
        self._segments = list(segments)
        self._seg_keys = list(seg_keys)
        self._leaf_keep.append(seg_arr)
        return seg_arr

    def relower(self, query: QueryContext, id_sets=None) -> "CPlan":
        """This plan for `query`, a query of the same shape (query_shape: only the filter's literals differ): the
        aggregations, keys, ORDER BY / trim and sum bounds are shared, only the leaves are lowered again -- the
        per-segment predicate evaluators of the new literals (one pg_dict_id_sets launch per IN list)."""
        ops, preds = filter_program(query.filter)
        if len(preds) != len(self.leaf_preds):
            raise ValueError("relower: a query of another shape")
        new = copy.copy(self)
        new.query = query
        new.leaf_preds = preds
        seg_arr = new._lower_leaves(self.table, self._segments, self._seg_keys, preds, id_sets)
        p = abi.pg_plan.from_buffer_copy(self.plan)
        p.segments = seg_arr
        new.plan = p
        new._image = None
        new._image_lock = threading.Lock()
        new._tls = threading.local()
        return new

    @property
    def lowered(self) -> List[List[LoweredLeaf]]:
        """The lowered leaves as LoweredLeaf records, [segment][leaf] (built on first use: tests and bench.py's byte
        model read them; execution reads the pg_leaf table)."""
        if self._lowered is None:
            out = []
            L = len(self.leaf_preds)
            for si in range(len(self._segments)):
                row = []
                for li in range(L):
                    lw = self._per_seg.get((si, li))
                    if lw is None:
                        r = self._leaf_tab[si, li]
                        ids = None
                        n = int(r["num_ids"])
                        vec = self._vec[li]
                        if n and li in self._batch:
                            ids = np.array(self._batch[li][0][si, :n], dtype=np.int32)
                        elif n:
                            ids = np.array([int(vec["keep"][0][si])], dtype=np.int32)
                        lw = LoweredLeaf(int(r["kind"]), int(r["col_id"]), int(r["exclusive"]), int(r["lo"]),
                                         int(r["hi"]), ids)
                    row.append(lw)
                out.append(row)
            self._lowered = out
        return self._lowered

    def image(self, query_id: Optional[int] = None, deadline_ms: Optional[int] = None) -> Tuple[np.ndarray, int]:
        """The plan as one relocatable byte image (pg_image_header + arrays at offsets, include/pinot_gpu.h): what a
        Java GpuPlanMaker fills in a direct ByteBuffer, and its address.  Built once per plan; each calling thread gets
        its own copy, whose header carries the per-call scalars -- query id and deadline as passed here (default: the
        plan's own fields), flags and limits from the plan -- so two threads running one cached plan with different
        query ids or deadlines never see each other's values."""
        if self._image is None:
            with self._image_lock:
                if self._image is None:
                    regions = [a for a in self._keep + self._leaf_keep if isinstance(a, np.ndarray)]
                    self._image = abi.build_image(self.plan, self._leaf_tab, regions)
        t = self._tls
        if getattr(t, "image", None) is None:
            t.image = self._image.copy()
            t.header = abi.pg_image_header.from_buffer(t.image)
            t.addr = t.image.ctypes.data  # stable while the copy lives (ndarray.ctypes costs ~3 us a call)
        h, p = t.header, self.plan
        h.query_id = p.query_id if query_id is None else query_id
        h.deadline_ms = p.deadline_ms if deadline_ms is None else deadline_ms
        h.flags, h.limit = p.flags, p.limit
        h.num_groups_limit = p.num_groups_limit
        h.trim_threshold = min(p.trim_threshold, 0xFFFFFFFF)
        return t.image, t.addr

    @staticmethod
    def _batched_in_ids(preds, segments, seg_keys, cid, id_sets) -> dict:
        """{leaf: (ids [S, n], counts [S], literals widened to int64 / float64)} for the IN / NOT_IN leaves over numeric
        dictionaries of one stored type in every segment: the literals are coerced once (the first segment's dictionary
        type) and looked up in all segments by one id_sets call."""
        out = {}
        for li, p in enumerate(preds):
            if p.type not in ("IN", "NOT_IN"):
                continue
            cols = [s.columns.get(p.column) for s in segments]
            if any(c is None or c.dictionary is None for c in cols):
                continue
            d0 = cols[0].dictionary
            if d0.data_type not in ("INT", "LONG", "FLOAT", "DOUBLE") or \
                    any(c.dictionary.data_type != d0.data_type or c.dictionary.values.dtype != d0.values.dtype
                        for c in cols):
                continue
            lit = _coerced_literals(d0, p.values)
            if lit is None:
                continue
            ids, counts = id_sets(cid[p.column], d0.data_type, np.ascontiguousarray(lit), seg_keys)
            wide = np.ascontiguousarray(lit, dtype=np.int64 if d0.data_type in ("INT", "LONG") else np.float64)
            out[li] = (ids, counts, wide)
        return out
