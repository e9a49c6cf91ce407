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


_DELIM = re.compile(r"[,\t]")


class FileDataModel(GenericDataModel):
    """T/impl/model/file/FileDataModel.java: lines `user,item,pref[,ts]`
    (delimiter `,` or tab, :125,344), `#` comments and blank lines ignored
    (:399-401), optional transpose (:414-418), a repeated (user,item) keeps
    the LAST value (:511-527), and `user,item,` (empty pref) removes the
    preference (:424-450)."""

    def __init__(self, path, transpose=False):
        prefs = {}
        with open(path) as f:
            for line in f:
                line = line.rstrip("\n").rstrip("\r")
                if not line or line[0] == "#":
                    continue
                tok = _DELIM.split(line)
                u, it = int(tok[0]), int(tok[1])
                pref_s = tok[2] if len(tok) > 2 else ""
                has_ts = len(tok) > 3
                if transpose:
                    u, it = it, u
                if not has_ts and pref_s == "":
                    if u in prefs:
                        prefs[u].pop(it, None)
                        if not prefs[u]:
                            del prefs[u]
                    continue
                prefs.setdefault(u, {})[it] = float(np.float32(pref_s))
        super().__init__(prefs)
