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
