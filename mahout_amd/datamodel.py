"""DataModel inputs of the sketch path.

GenericDataModel / FileDataModel reduced to what CosineCM reads: the sorted
owner-ID universe and each owner's preferences sorted by key, in the SoA
layout of GenericUserPreferenceArray (long[] ids, float[] values,
T/impl/model/GenericUserPreferenceArray.java:52-54) -- here one CSR
(offsets, keys, values) over all owners, which is exactly what
cms_ingest_csr consumes.
"""
import re

import numpy as np


class NoSuchUserException(KeyError):
    """org.apache.mahout.cf.taste.common.NoSuchUserException"""


class GenericDataModel:
    """T/impl/model/GenericDataModel.java:80-137: per-user preferences sorted
    by item (:91), item IDs sorted (:120), user IDs sorted (:134)."""

    def __init__(self, user_prefs):
        # user_prefs: {userID: {itemID: float}}
        self.user_ids = np.array(sorted(user_prefs), dtype=np.int64)
        items = set()
        offsets = [0]
        keys, vals = [], []
        for u in self.user_ids:
            prefs = user_prefs[int(u)]
            for it in sorted(prefs):
                keys.append(it)
                vals.append(np.float32(prefs[it]))
                items.add(it)
            offsets.append(len(keys))
        self.item_ids = np.array(sorted(items), dtype=np.int64)
        self.offsets = np.array(offsets, dtype=np.int64)
        self.keys = np.array(keys, dtype=np.int64)
        self.values = np.array(vals, dtype=np.float32)

    @classmethod
    def from_csr(cls, user_ids, offsets, keys, values):
        self = cls.__new__(cls)
        self.user_ids = np.ascontiguousarray(user_ids, np.int64)
        self.offsets = np.ascontiguousarray(offsets, np.int64)
        self.keys = np.ascontiguousarray(keys, np.int64)
        self.values = None if values is None else np.ascontiguousarray(values, np.float32)
        self.item_ids = np.unique(self.keys)
        return self

    def getUserIDs(self):
        return self.user_ids

    def getItemIDs(self):
        return self.item_ids

    def getNumUsers(self):
        return int(self.user_ids.size)

    def getNumItems(self):
        return int(self.item_ids.size)

    def hasPreferenceValues(self):
        return self.values is not None

    def getMinPreference(self):
        """Smallest preference value (GenericDataModel.java:87-116); +inf when
        empty; NaN without values (AbstractDataModel.java:31-34)."""
        if self.values is None:
            return float("nan")
        return float(self.values.min()) if self.values.size else float("inf")

    def getMaxPreference(self):
        if self.values is None:
            return float("nan")
        return float(self.values.max()) if self.values.size else float("-inf")

    def getPreferenceValue(self, user_id, item_id):
        """GenericDataModel.getPreferenceValue (:244-253): the value, or None."""
        keys, vals = self.getPreferencesFromUser(user_id)
        j = np.searchsorted(keys, item_id)
        if j < keys.size and keys[j] == item_id:
            return None if vals is None else float(vals[j])
        return None

    def getPreferencesFromUser(self, user_id):
        """(item IDs ascending, float values) -- GenericDataModel.java:210-216."""
        i = np.searchsorted(self.user_ids, user_id)
        if i >= self.user_ids.size or self.user_ids[i] != user_id:
            raise NoSuchUserException(user_id)
        lo, hi = self.offsets[i], self.offsets[i + 1]
        v = None if self.values is None else self.values[lo:hi]
        return self.keys[lo:hi], v


_JAVA_DEC = re.compile(r"[+-]?(?:NaN|Infinity|(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?[fFdD]?)")
_JAVA_HEX = re.compile(r"([+-]?)0[xX]([0-9a-fA-F]*)\.?([0-9a-fA-F]*)[pP]([+-]?\d+)[fFdD]?")
_LONG = re.compile(r"[+-]?\d+")


def _round_to_f32(q):
    """The float32 nearest the exact rational q (ties to even), as IEEE 754
    round-to-nearest does for Float.parseFloat (JLS: "rounded to type float
    by the usual round-to-nearest rule")."""
    from fractions import Fraction
    try:
        x = float(q)  # correctly rounded to double (int / int true division)
    except OverflowError:
        return np.float32(np.inf if q > 0 else -np.inf)
    with np.errstate(over="ignore", under="ignore"):
        f = np.float32(x)
    if float(f) == x:  # q is within half a double ulp of a float32: that one
        return f
    # decimal -> double -> float rounds twice; only a double that lands
    # exactly on a float32 midpoint can end on the wrong side: resolve it from q
    up = x > float(f) if np.isfinite(f) else x < 0
    if not np.isfinite(f):  # x beyond FLT_MAX: f is inf, its neighbour FLT_MAX
        g = np.float32(np.finfo(np.float32).max) * np.float32(1 if x > 0 else -1)
        f, g = g, f
        up = not up
    with np.errstate(over="ignore"):
        g = np.nextafter(f, np.float32(np.inf) if up else np.float32(-np.inf))
    gv = Fraction(float(g)) if np.isfinite(g) else Fraction(2 ** 128) * (1 if up else -1)
    mid = (Fraction(float(f)) + gv) / 2
    if Fraction(x) != mid:
        return np.float32(f) if abs(Fraction(x) - Fraction(float(f))) < abs(Fraction(x) - gv) else g
    if q == mid:  # an exact tie: the even significand (inf counts as even past FLT_MAX)
        return f if (int(np.float32(f).view(np.uint32)) & 1) == 0 else g
    return g if (q > mid) == up else f


_F32_CACHE = {}


def java_parse_float(s):
    """java.lang.Float.parseFloat: surrounding whitespace (chars <= ' ')
    trimmed, optional sign, NaN / Infinity, decimal or hexadecimal
    significand, optional f/F/d/D suffix; the exact value rounded once to
    float32.  Raises ValueError (NumberFormatException) otherwise."""
    r = _F32_CACHE.get(s)
    if r is not None:
        return r
    from fractions import Fraction
    t = s.strip("".join(chr(c) for c in range(33)))
    if _JAVA_DEC.fullmatch(t):
        body = t.rstrip("fFdD") if t[-1:] in "fFdD" and "Infinity" not in t else t
        neg = body.startswith("-")
        core = body.lstrip("+-")
        if core == "NaN":
            r = np.float32(np.nan)
        elif core == "Infinity":
            r = np.float32(-np.inf if neg else np.inf)
        else:
            q = Fraction(core)
            r = _round_to_f32(-q if neg else q)
            if neg and r == 0:
                r = np.float32(-0.0)
    else:
        m = _JAVA_HEX.fullmatch(t)
        if not m or not (m.group(2) or m.group(3)):
            raise ValueError(f"For input string: \"{s}\"")
        digits = (m.group(2) or "") + (m.group(3) or "")
        q = Fraction(int(digits, 16), 16 ** len(m.group(3) or "")) * Fraction(2) ** int(m.group(4))
        r = _round_to_f32(-q if m.group(1) == "-" else q)
        if m.group(1) == "-" and r == 0:
            r = np.float32(-0.0)
    if len(_F32_CACHE) < 65536:
        _F32_CACHE[s] = r
    return r


def java_parse_long(s):
    """java.lang.Long.parseLong (FileDataModel.readUserIDFromString /
    readItemIDFromString): decimal digits with an optional sign, no
    whitespace, within the long range; ValueError otherwise."""
    if not _LONG.fullmatch(s):
        raise ValueError(f"For input string: \"{s}\"")
    v = int(s)
    if not -2 ** 63 <= v < 2 ** 63:
        raise ValueError(f"For input string: \"{s}\"")
    return v


class FileDataModel(GenericDataModel):
    """T/impl/model/file/FileDataModel.java, one data file, no update files:

    - the delimiter is ',' if the first data line (blank and '#' lines
      skipped) holds one, else tab (determineDelimiter, :344-352); every
      line is split on that single character, empty tokens kept (Guava
      Splitter.on, :201);
    - the file has preference values when that first line has a non-empty
      third token (:210-214); otherwise it is a boolean model
      (processLineWithoutID, :560-603; hasPreferenceValues() is false);
    - IDs are Long.parseLong, values Float.parseFloat (:411-412, :455);
    - transpose swaps user and item (:414-418);
    - a repeated (user, item) keeps the LAST value (:511-527);
    - `user,item,` (empty value, no timestamp) removes the preference
      (:493-508) -- the user stays in the model even with no preferences left
      (GenericDataModel.toDataMap keeps the emptied collection, :160-168).
    """

    def __init__(self, path, transpose=False):
        with open(path) as f:
            lines = [ln.rstrip("\n").rstrip("\r") for ln in f]
        first = next((ln for ln in lines if ln and ln[0] != "#"), None)
        if first is None:
            raise ValueError("dataFile is empty")
        if "," in first:
            delim = ","
        elif "\t" in first:
            delim = "\t"
        else:
            raise ValueError("Did not find a delimiter in first line")
        ftok = first.split(delim)
        has_values = len(ftok) >= 3 and ftok[2] != ""
        prefs = {}
        for line in lines:
            if not line or line[0] == "#":
                continue
            tok = line.split(delim)
            if len(tok) < 2 or (has_values and len(tok) < 3):
                raise ValueError(f"NoSuchElementException: too few fields in line {line!r}")
            u, it = java_parse_long(tok[0]), java_parse_long(tok[1])
            has_pref = len(tok) >= 3
            pref_s = tok[2] if has_pref else ""
            has_ts = len(tok) >= 4
            if transpose:
                u, it = it, u
            if (has_values or has_pref) and not has_ts and pref_s == "":
                if u in prefs:
                    prefs[u].pop(it, None)
                continue
            if has_values:
                prefs.setdefault(u, {})[it] = float(java_parse_float(pref_s))
            else:
                prefs.setdefault(u, {})[it] = 1.0
        super().__init__(prefs)
        if not has_values:
            self.values = None  # GenericBooleanPrefDataModel
