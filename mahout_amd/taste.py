"""Host-side mirror of the reference's plugin surface for the sketch path.

``CosineCM`` keeps the names, argument meaning and error behaviour of
org.apache.mahout.cf.taste.impl.similarity.CosineCM
(T/impl/similarity/CosineCM.java) and of the two plugin interfaces it
serves, UserSimilarity (T/similarity/UserSimilarity.java:31-58) and
ItemSimilarity (T/similarity/ItemSimilarity.java:31-64); every similarity
is computed by libmahout_cms.so on the GPU.

Shape: the reference sizes each owner's sketch from CountMinSketchConfig's
(delta, epsilon) (CosineCM.java:63,86).  ``CountMinSketchConfig`` keeps that
per-owner mode (u1 hashed at u2's shape on the GPU).  The fixed-shape configs of this
path (d, w for every owner) are expressed by ``FixedShapeConfig``, whose
getDelta/getEpsilon return exp(-d) and e/w -- the subclass override the
reference allows (CountMinSketchConfig.getDelta/getEpsilon are public,
non-final) -- and the shape actually used is the one
AbstractCountMinSketch(delta, epsilon) derives from them.
"""
import math

import numpy as np

from . import _lib
from .datamodel import NoSuchUserException
from .sketch import SketchTable, frac_bits_for, shape_from_delta_epsilon


class TasteException(Exception):
    """org.apache.mahout.cf.taste.common.TasteException"""


class NoSuchItemException(TasteException, KeyError):
    """org.apache.mahout.cf.taste.common.NoSuchItemException"""


class Weighting:
    UNWEIGHTED = "UNWEIGHTED"
    WEIGHTED = "WEIGHTED"


class HashFunctionBuilder:
    """HashFunctionBuilder(long seed) (T/impl/common/HashFunctionBuilder.java:23-29)."""

    def __init__(self, seed):
        self.seed = int(seed)


class FixedShapeConfig:
    """Every owner gets the same (depth, width)."""

    def __init__(self, depth, width):
        self.depth = int(depth)
        self.width = int(width)

    def getDelta(self, owner_id=None):
        return math.exp(-float(self.depth))

    def getEpsilon(self, owner_id=None):
        return math.e / float(self.width)

    def shape(self):
        """(width, depth) that new DoubleCountMinSketch(delta, epsilon, ...) builds."""
        return shape_from_delta_epsilon(self.getDelta(), self.getEpsilon())


class CountMinSketchConfig:
    """CountMinSketchConfig(q) (T/impl/common/CountMinSketchConfig.java:57-60):
    per-owner (delta, epsilon) chosen by the Fmeasure search.  configure()
    runs computeConfig (:120-158) on the GPU when the CosineCM that owns the
    data is built; setConfig() takes (delta, epsilon) arrays computed
    elsewhere (the ser/ cache of :74-95 in the reference).  getDelta /
    getEpsilon before configuration raise TasteException, as :230-251 do."""

    def __init__(self, q):
        self.q = float(q)
        self._explicit = None
        self._result = None  # (owner ids, delta, epsilon) once configured

    def setConfig(self, delta, epsilon):
        self._explicit = (np.asarray(delta, np.float64), np.asarray(epsilon, np.float64))

    def _configure(self, table, dataModel):
        if self._explicit is not None:
            table.set_owner_delta_epsilon(*self._explicit)
        else:
            table.configure_owner_shapes(self.q, dataModel.getNumItems())
        de, ep, _, _ = table.owner_shapes()
        self._result = (dataModel.getUserIDs(), de, ep)

    def _lookup(self, arr, userID):
        if self._result is None:
            raise TasteException("delta is null, call configure method first")
        ids = self._result[0]
        i = np.searchsorted(ids, userID)
        return float(arr[i]) if i < ids.size and ids[i] == userID else 0.0  # trove: missing key -> 0.0

    def getDelta(self, userID):
        return self._lookup(self._result[1] if self._result else None, userID)

    def getEpsilon(self, userID):
        return self._lookup(self._result[2] if self._result else None, userID)


def counter_units(offsets, values):
    """(frac_bits, counters) for a DataModel: exact u32 counters in units of
    2^-frac_bits when every preference is a non-negative multiple of
    2^-frac_bits and every owner's total stays below 2^32 such units (the
    integer fast paths, bit-identical similarities); otherwise
    DoubleCountMinSketch's own fp64 counters, filled in DataModel order."""
    if values is None:
        return 0, "u32"
    v = np.asarray(values, np.float32)
    if v.size and (not np.all(np.isfinite(v)) or (v < 0).any()):
        return 0, "f64"
    try:
        fb = frac_bits_for(v)
    except ValueError:
        return 0, "f64"
    off = np.asarray(offsets, np.int64)
    if v.size:
        mass = np.add.reduceat(np.ldexp(v.astype(np.float64), fb), off[:-1].clip(max=v.size - 1))
        mass[off[1:] == off[:-1]] = 0.0
        if (mass >= 2.0 ** 32).any():
            return 0, "f64"
    return fb, "u32"


def _map_error(e, owner_kind="user"):
    if e.code == _lib.CMS_E_NO_SUCH_ID:
        return NoSuchUserException(str(e)) if owner_kind == "user" else NoSuchItemException(str(e))
    if e.code in (_lib.CMS_E_PARAM, _lib.CMS_E_SHAPE):
        return ValueError(str(e))  # IllegalArgumentException
    return TasteException(str(e))


class CosineCM:
    """CosineCM(DataModel, [Weighting,] CountMinSketchConfig, HashFunctionBuilder).

    Owners are the DataModel's users (sketches keyed by item ID).  Over a
    transposed DataModel the owners are items and userSimilarity /
    itemSimilarity are the sketch-cosine ItemSimilarity.
    """

    def __init__(self, dataModel, conf, hfBuilder, weighting=Weighting.UNWEIGHTED, device=-1):
        if not dataModel.hasPreferenceValues():  # CosineCM.java:38
            raise ValueError("DataModel doesn't have preference values")
        self._per_owner = isinstance(conf, CountMinSketchConfig)
        if self._per_owner:
            width = depth = None  # each owner has its own shape
        else:
            width, depth = conf.shape() if hasattr(conf, "shape") else (conf.width, conf.depth)
        self._model = dataModel
        self._conf = conf
        self._hfb = hfBuilder
        self._weighted = weighting == Weighting.WEIGHTED
        self._device = device
        self.depth, self.width = depth, width
        self._inferrer = None
        self._build()

    def _build(self):
        m = self._model
        fb, counters = counter_units(m.offsets, m.values)
        try:
            if self._per_owner:
                self._table = SketchTable(m.getNumUsers(), seed=self._hfb.seed, weighted=self._weighted,
                                          device=self._device, owner_ids=m.getUserIDs(), per_owner=True,
                                          frac_bits=fb, counters=counters)
                self._table.ingest_csr(m.offsets, m.keys, m.values)
                self._conf._configure(self._table, m)
            else:
                self._table = SketchTable(m.getNumUsers(), depth=self.depth, width=self.width, seed=self._hfb.seed,
                                          weighted=self._weighted, device=self._device, owner_ids=m.getUserIDs(),
                                          frac_bits=fb, counters=counters)
                self._table.ingest_csr(m.offsets, m.keys, m.values)
            self._table.finalize()
        except _lib.CmsError as e:
            raise _map_error(e)

    @property
    def table(self):
        return self._table

    # ---- UserSimilarity ----
    def userSimilarity(self, userID1, userID2):
        try:
            return self._table.similarity(userID1, userID2)
        except _lib.CmsError as e:
            raise _map_error(e, "user")

    def setPreferenceInferrer(self, inferrer):
        if inferrer is None:
            raise ValueError("inferrer is null")
        self._inferrer = inferrer  # unused by the sketch cosine, as in CosineCM

    # ---- ItemSimilarity (owners are items in the transposed orientation) ----
    def itemSimilarity(self, itemID1, itemID2):
        try:
            return self._table.similarity(itemID1, itemID2)
        except _lib.CmsError as e:
            raise _map_error(e, "item")

    def itemSimilarities(self, itemID1, itemID2s):
        try:
            return self._table.similarities(itemID1, itemID2s)
        except _lib.CmsError as e:
            raise _map_error(e, "item")

    def allSimilarItemIDs(self, itemID):
        """AbstractItemSimilarity.allSimilarItemIDs: every owner whose
        similarity is not NaN (T/impl/similarity/AbstractItemSimilarity.java:48-58)."""
        ids = self._model.getUserIDs()
        sims = self.itemSimilarities(itemID, ids)
        return ids[~np.isnan(sims)]

    # ---- recommender-side consumers ----
    def mostSimilarUserIDs(self, userID, howMany):
        """GenericUserBasedRecommender.mostSimilarUserIDs (:119-127) with
        TopItems.getTopUsers (TopItems.java:91-136)."""
        if howMany < 1:
            raise ValueError("howMany must be at least 1")
        try:
            ids, _ = self._table.most_similar(userID, howMany)
        except _lib.CmsError as e:
            raise _map_error(e, "user")
        return ids

    def getExportedCMProfileEstimate(self, userID, itemID):
        """DoubleCountMinSketch.get(itemID) on userID's sketch, the point query
        GenericUserBasedRecommender.doEstimatePreference uses (:153-158)."""
        try:
            return self._table.point_query(userID, itemID)
        except _lib.CmsError as e:
            raise _map_error(e, "user")

    def refresh(self, alreadyRefreshed=None):
        """Refreshable.refresh: rebuild every sketch from the data model."""
        self._table.close()
        self._build()

    def close(self):
        self._table.close()


class NearestNUserNeighborhood:
    """NearestNUserNeighborhood(n, similarity, model): the n most similar
    users (T/impl/neighborhood/NearestNUserNeighborhood.java) -- TopItems
    .getTopUsers with minSimilarity -inf and sampling rate 1, i.e. the same
    order as mostSimilarUserIDs."""

    def __init__(self, n, userSimilarity, dataModel):
        if n < 1:
            raise ValueError("n must be at least 1")
        self.n = n
        self._sim = userSimilarity
        self._model = dataModel

    def getUserNeighborhood(self, userID):
        return self._sim.mostSimilarUserIDs(userID, self.n)

    def getUserNeighborhoods(self, userIDs):
        """getUserNeighborhood for many users: (offsets, neighbour IDs) from
        one all-owners top-n pass (cms_top_k_all: the same lists as
        mostSimilarUserIDs, each unordered pair scored once)."""
        table = self._sim.table
        ids, _, cnt = table.top_k_all(self.n)
        owners = self._model.getUserIDs()
        users = np.ascontiguousarray(userIDs, np.int64)
        rows = np.searchsorted(owners, users)
        if np.any(rows >= owners.size) or np.any(owners[np.minimum(rows, owners.size - 1)] != users):
            bad = users[(rows >= owners.size) | (owners[np.minimum(rows, owners.size - 1)] != users)][0]
            raise NoSuchUserException(int(bad))
        c = cnt[rows].astype(np.int64)
        off = np.zeros(users.size + 1, np.int64)
        np.cumsum(c, out=off[1:])
        sel = ids[rows]
        nb = sel[np.arange(self.n)[None, :] < c[:, None]]
        return off, np.ascontiguousarray(nb, np.int64)


class GenericUserBasedRecommender:
    """GenericUserBasedRecommender(model, neighborhood, CosineCM): the
    estimate path with the sketch point query
    (T/impl/recommender/GenericUserBasedRecommender.java:108-116, 134-184),
    capped by EstimatedPreferenceCapper when the model has min/max (:209-216)."""

    def __init__(self, dataModel, neighborhood, similarity):
        self._model = dataModel
        self._nb = neighborhood
        self._sim = similarity
        lo, hi = dataModel.getMinPreference(), dataModel.getMaxPreference()
        self._capper = None if (np.isnan(lo) and np.isnan(hi)) else (lo, hi)

    def estimatePreference(self, userID, itemID):
        actual = self._model.getPreferenceValue(userID, itemID)
        if actual is not None:
            return np.float32(actual)
        return self.doEstimatePreferences(userID, self._nb.getUserNeighborhood(userID), [itemID])[0]

    def doEstimatePreferences(self, theUserID, theNeighborhood, itemIDs):
        """doEstimatePreference for many items at once (one GPU launch)."""
        if len(theNeighborhood) == 0:
            return np.full(len(itemIDs), np.nan, np.float32)
        try:
            return self._sim.table.estimate_preferences(theUserID, theNeighborhood, itemIDs, self._capper)
        except _lib.CmsError as e:
            raise _map_error(e, "user")

    def getAllOtherItems(self, theNeighborhood, theUserID, includeKnownItems=False):
        """getAllOtherItems (GenericUserBasedRecommender.java:187-198): the
        neighbours' items as a FastIDSet, the user's own removed."""
        possible = FastIDSet()
        for u in theNeighborhood:
            possible.addAll(self._item_set(u))
        if not includeKnownItems:
            possible.removeAll(self._item_set(theUserID))
        return possible

    def _item_set(self, userID):
        """GenericDataModel.getItemIDsFromUser (GenericDataModel.java:219-227)."""
        keys, _ = self._model.getPreferencesFromUser(userID)
        s = FastIDSet(len(keys))
        for k in keys.tolist():
            s.add(k)
        return s

    def _model_csr(self):
        """The DataModel as (user IDs ascending, offsets, item IDs in
        getPreferencesFromUser order), built once."""
        if getattr(self, "_csr", None) is None:
            m = self._model
            if all(hasattr(m, a) for a in ("user_ids", "offsets", "keys")):
                self._csr = (m.user_ids, m.offsets, m.keys)
            else:
                uids = np.asarray(m.getUserIDs(), np.int64)
                parts = [np.asarray(m.getPreferencesFromUser(int(u))[0], np.int64) for u in uids]
                off = np.zeros(uids.size + 1, np.int64)
                np.cumsum([p.size for p in parts], out=off[1:])
                self._csr = (uids, off, np.concatenate(parts) if parts else np.zeros(0, np.int64))
        return self._csr

    def recommend_all(self, userIDs, howMany, includeKnownItems=False):
        """recommend(userID, howMany) for every user of userIDs in one native
        call (cms_recommend_batch): the neighbourhoods from one all-owners
        top-n pass, the candidates in FastIDSet order and TopItems.getTopItems
        on the host side of the library, every estimate in one device batch.
        Returns one [(itemID, float value)] list per user, equal to recommend()."""
        if howMany < 1:
            raise ValueError("howMany must be at least 1")
        users = np.ascontiguousarray(userIDs, np.int64)
        nb_off, nb = self._nb.getUserNeighborhoods(users)
        mu, po, pi = self._model_csr()
        try:
            cnt, items, vals = self._sim.table.recommend_batch(users, nb_off, nb, mu, po, pi, howMany,
                                                               includeKnownItems, self._capper)
        except _lib.CmsError as e:
            raise _map_error(e, "user")
        return [[(int(items[u, j]), vals[u, j]) for j in range(int(cnt[u]))] for u in range(users.size)]

    def recommend(self, userID, howMany, includeKnownItems=False):
        """recommend(userID, howMany) (GenericUserBasedRecommender.java:84-105):
        the neighbourhood, the candidate items in FastIDSet iteration order,
        their estimates (one GPU call), then TopItems.getTopItems
        (TopItems.java:47-88) -- a JDK PriorityQueue under the reversed
        ByValueRecommendedItemComparator and a stable sort, so tied values
        come out in the reference's order.  [(itemID, float value)]."""
        if howMany < 1:
            raise ValueError("howMany must be at least 1")
        nb = self._nb.getUserNeighborhood(userID)
        if len(nb) == 0:
            return []
        items = self.getAllOtherItems(nb, userID, includeKnownItems).toList()
        est = self.doEstimatePreferences(userID, nb, items) if items else np.zeros(0, np.float32)
        return get_top_items(howMany, items, est)


def _is_prime(n):
    """Primality of n < 2^63 (deterministic Miller-Rabin bases)."""
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _next_prime(n):
    """commons-math3 Primes.nextPrime(n): the smallest prime >= n."""
    n = max(n, 2)
    while not _is_prime(n):
        n += 1
    return n


def next_twin_prime(n):
    """RandomUtils.nextTwinPrime (math/.../common/RandomUtils.java:86-98): the
    larger of the first twin-prime pair whose smaller member is >= n."""
    if n > 2147482949:
        raise ValueError(n)
    if n <= 3:
        return 5
    nxt = _next_prime(n)
    while not _is_prime(nxt + 2):
        nxt = _next_prime(nxt + 4)
    return nxt + 2


class FastIDSet:
    """T/impl/common/FastIDSet.java: open addressing with double hashing
    (hash = (int) key & 0x7FFFFFFF, jump = 1 + hash % (size - 2)), REMOVED
    markers, twin-prime table sizes and float load-factor arithmetic -- what
    fixes its iteration order (the order TopItems.getTopItems sees the
    candidates in, hence the order of tied recommendations)."""

    NULL = -(1 << 63)
    REMOVED = (1 << 63) - 1

    def __init__(self, size=2, loadFactor=1.5):
        self.lf = np.float32(loadFactor)
        self.keys = [self.NULL] * next_twin_prime(int(self.lf * np.float32(size)))
        self.numEntries = 0
        self.numSlotsUsed = 0

    def _probe(self, key, for_add):
        h = (key & 0xFFFFFFFF) & 0x7FFFFFFF  # (int) key & 0x7FFFFFFF
        keys = self.keys
        n = len(keys)
        jump = 1 + h % (n - 2)
        index = h % n
        cur = keys[index]
        if not for_add:
            while cur != self.NULL and key != cur:
                index -= jump - n if index < jump else jump
                cur = keys[index]
            return index
        while cur != self.NULL and cur != self.REMOVED and key != cur:
            index -= jump - n if index < jump else jump
            cur = keys[index]
        if cur != self.REMOVED:
            return index
        add_index = index
        while cur != self.NULL and key != cur:
            index -= jump - n if index < jump else jump
            cur = keys[index]
        return index if key == cur else add_index

    def add(self, key):
        key = int(key)
        if np.float32(self.numSlotsUsed) * self.lf >= np.float32(len(self.keys)):
            if np.float32(self.numEntries) * self.lf >= np.float32(self.numSlotsUsed):
                self._rehash(next_twin_prime(int(self.lf * np.float32(len(self.keys)))))
            else:
                self._rehash(next_twin_prime(int(self.lf * np.float32(self.numEntries))))
        index = self._probe(key, True)
        old = self.keys[index]
        if old != key:
            self.keys[index] = key
            self.numEntries += 1
            if old == self.NULL:
                self.numSlotsUsed += 1
            return True
        return False

    def remove(self, key):
        key = int(key)
        if key in (self.NULL, self.REMOVED):
            return False
        index = self._probe(key, False)
        if self.keys[index] == self.NULL:
            return False
        self.keys[index] = self.REMOVED
        self.numEntries -= 1
        return True

    def _rehash(self, new_size):
        old = self.keys
        self.numEntries = 0
        self.numSlotsUsed = 0
        self.keys = [self.NULL] * new_size
        for k in old:
            if k != self.NULL and k != self.REMOVED:
                self.add(k)

    def _live(self):
        return [k for k in self.keys if k != self.NULL and k != self.REMOVED]

    def addAll(self, other):
        changed = False
        for k in other._live():
            changed |= self.add(k)
        return changed

    def removeAll(self, other):
        changed = False
        for k in other._live():
            changed |= self.remove(k)
        return changed

    def toList(self):
        """Iteration order (KeyIterator: table positions, NULL and REMOVED skipped)."""
        return self._live()

    def __len__(self):
        return self.numEntries


def _cmp_by_value_reversed(a, b):
    """Collections.reverseOrder(ByValueRecommendedItemComparator): the queue
    head is the lowest float value (ByValueRecommendedItemComparator.java:37-41)."""
    return -1 if a[1] < b[1] else 1 if a[1] > b[1] else 0


def get_top_items(howMany, itemIDs, estimates):
    """TopItems.getTopItems (TopItems.java:47-88) with no rescorer: a
    PriorityQueue of howMany + 1, items kept while their (double) estimate
    beats the head once full, then the queue's array order stably sorted by
    float value descending.  [(itemID, float32 value)]."""
    q = _JavaPriorityQueue(_cmp_by_value_reversed)
    full = False
    lowest = float("-inf")
    for item, e in zip(itemIDs, estimates):
        pref = float(e)
        if pref != pref or (full and not pref > lowest):
            continue
        q.add((int(item), np.float32(pref)))
        if full:
            q.poll()
        elif len(q) > howMany:
            full = True
            q.poll()
        lowest = float(q.peek()[1])
    out = list(q.q)
    out.sort(key=lambda x: -float(x[1]))  # Collections.sort is stable, as is list.sort
    return out


# ---- the precomputed-similarity consumer ----------------
# GenericItemSimilarity(Iterable<ItemItemSimilarity>) is how Taste consumes
# precomputed item-item similarities (T/impl/similarity/GenericItemSimilarity.java:71-95,
# 172-236); the all-pairs lists of cms_top_k_all / cms_top_k_refresh feed it
# through ``similarities_from_top_k``.

class ItemItemSimilarity:
    """GenericItemSimilarity.ItemItemSimilarity (:251-315): value must lie in
    [-1, 1] (NaN rejected, as Preconditions.checkArgument does, :264-266)."""

    __slots__ = ("itemID1", "itemID2", "value")

    def __init__(self, itemID1, itemID2, value):
        value = float(value)
        if not (-1.0 <= value <= 1.0):
            raise ValueError("Illegal value: %r. Must be: -1.0 <= value <= 1.0" % value)
        self.itemID1 = int(itemID1)
        self.itemID2 = int(itemID2)
        self.value = value

    def getItemID1(self):
        return self.itemID1

    def getItemID2(self):
        return self.itemID2

    def getValue(self):
        return self.value

    def __repr__(self):
        return "ItemItemSimilarity[%d,%d:%r]" % (self.itemID1, self.itemID2, self.value)


def _cmp_item_item(a, b):
    """ItemItemSimilarity.compareTo (:296-300): highest value first."""
    return -1 if a.value > b.value else 1 if a.value < b.value else 0


class _JavaPriorityQueue:
    """java.util.PriorityQueue with a comparator: a binary min-heap with the
    JDK's siftUp / siftDown (offer, poll, peek), so ties leave the queue in
    the same order the reference's does."""

    def __init__(self, cmp):
        self.q = []
        self.cmp = cmp

    def add(self, x):
        q, cmp = self.q, self.cmp
        k = len(q)
        q.append(x)
        while k > 0:  # siftUpUsingComparator
            parent = (k - 1) >> 1
            e = q[parent]
            if cmp(x, e) >= 0:
                break
            q[k] = e
            k = parent
        q[k] = x

    def peek(self):
        return self.q[0]

    def poll(self):
        q, cmp = self.q, self.cmp
        result = q[0]
        x = q.pop()
        n = len(q)
        if n:
            k, half = 0, n >> 1
            while k < half:  # siftDownUsingComparator
                child = 2 * k + 1
                c = q[child]
                right = child + 1
                if right < n and cmp(c, q[right]) > 0:
                    child = right
                    c = q[child]
                if cmp(x, c) <= 0:
                    break
                q[k] = c
                k = child
            q[k] = x
        return result

    def __len__(self):
        return len(self.q)


def get_top_item_item_similarities(howMany, allSimilarities):
    """TopItems.getTopItemItemSimilarities (T/impl/recommender/TopItems.java:145-174):
    a PriorityQueue in reverse compareTo order (lowest value at the head), a
    strict '>' admission once full, then Collections.sort (stable) of the
    queue's array order."""
    import functools
    pq = _JavaPriorityQueue(lambda a, b: -_cmp_item_item(a, b))  # Collections.reverseOrder()
    full = False
    lowest = -math.inf
    for s in allSimilarities:
        v = s.value
        if not math.isnan(v) and (not full or v > lowest):
            pq.add(s)
            if full:
                pq.poll()
            elif len(pq) > howMany:
                full = True
                pq.poll()
            lowest = pq.peek().value
    result = list(pq.q)
    result.sort(key=functools.cmp_to_key(_cmp_item_item))  # stable, as Collections.sort
    return result


class GenericItemSimilarity:
    """org.apache.mahout.cf.taste.impl.similarity.GenericItemSimilarity over
    precomputed similarities: ordered (smaller ID first) pair map where a later
    value wins, a pair of an item with itself skipped (assumed 1.0), and the
    per-item index of similar items (:172-205)."""

    def __init__(self, similarities, maxToKeep=None):
        if maxToKeep is not None:
            similarities = get_top_item_item_similarities(int(maxToKeep), similarities)
        self._maps = {}
        self._index = {}
        for s in similarities:
            a, b = s.itemID1, s.itemID2
            if a == b:
                continue
            lo, hi = (a, b) if a < b else (b, a)
            self._maps.setdefault(lo, {})[hi] = s.value
            self._index.setdefault(lo, set()).add(hi)
            self._index.setdefault(hi, set()).add(lo)

    @classmethod
    def from_similarity(cls, otherSimilarity, itemIDs, maxToKeep=None):
        """GenericItemSimilarity(ItemSimilarity, DataModel[, maxToKeep])
        (:126-160): every pair i < j of the item IDs in ascending order, NaN
        pairs skipped, as DataModelSimilaritiesIterator enumerates them
        (:317-353); one batched itemSimilarities call per item on the GPU."""
        ids = [int(x) for x in sorted(itemIDs)]

        def pairs():
            for i, a in enumerate(ids[:-1]):
                rest = ids[i + 1:]
                vals = otherSimilarity.itemSimilarities(a, rest)
                for b, v in zip(rest, vals):
                    if not math.isnan(v):  # the iterator skips NaN pairs (:341)
                        yield ItemItemSimilarity(a, b, v)
        return cls(pairs(), maxToKeep)

    def itemSimilarity(self, itemID1, itemID2):
        """(:219-236): 1.0 for an item with itself, NaN for a pair never given."""
        if itemID1 == itemID2:
            return 1.0
        lo, hi = (itemID1, itemID2) if itemID1 < itemID2 else (itemID2, itemID1)
        return self._maps.get(lo, {}).get(hi, math.nan)

    def itemSimilarities(self, itemID1, itemID2s):
        return np.array([self.itemSimilarity(itemID1, int(b)) for b in itemID2s], np.float64)

    def allSimilarItemIDs(self, itemID):
        """(:248-251).  The reference returns its FastIDSet's hash order; this
        returns the same IDs in ascending order (order unpinned)."""
        return np.array(sorted(self._index.get(int(itemID), ())), np.int64)

    def refresh(self, alreadyRefreshed=None):
        pass  # (:254-256) does nothing


def similarities_from_top_k(ids, scores, counts, owner_ids=None):
    """ItemItemSimilarity records of the all-pairs lists (cms_top_k_all /
    cms_top_k_refresh: [n][k] partner IDs and scores, counts[n]) in owner order
    then list order -- the iterable GenericItemSimilarity(Iterable) takes."""
    n = len(counts)
    for r in range(n):
        a = int(owner_ids[r]) if owner_ids is not None else r
        for i in range(int(counts[r])):
            yield ItemItemSimilarity(a, int(ids[r, i]), float(scores[r, i]))
