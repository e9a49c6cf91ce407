/*
 * Drop-in for the CosineCM sketch-cosine path (reference:
 * mr/src/main/java/org/apache/mahout/cf/taste/impl/similarity/CosineCM.java)
 * backed by libmahout_cms.so (include/mahout_cms.h) through the JNI shim in
 * integration/jni/mahout_cms_jni.c.
 *
 * NOTE: written against the reference's Taste interfaces; no JDK exists in
 * the build image, so this file is not compiled here (see INTEGRATION.md).
 *
 * Shape: either every owner gets the same (depth, width) -- the fixed-shape
 * configs of this path -- or, as the reference does, each owner is sized by a
 * CountMinSketchConfig (per-owner (delta, epsilon); CosineCM.java:26-39,83-96):
 * the config's getDelta/getEpsilon values are handed to the library once, or
 * the Fmeasure search itself runs on the GPU (the q constructor).
 */
package org.apache.mahout.cf.taste.impl.similarity;

import java.util.ArrayList;
import java.util.Collection;
import java.util.List;
import java.util.concurrent.locks.ReentrantReadWriteLock;

import org.apache.mahout.cf.taste.common.NoSuchItemException;
import org.apache.mahout.cf.taste.common.NoSuchUserException;
import org.apache.mahout.cf.taste.common.Refreshable;
import org.apache.mahout.cf.taste.common.TasteException;
import org.apache.mahout.cf.taste.common.Weighting;
import org.apache.mahout.cf.taste.impl.common.CountMinSketchConfig;
import org.apache.mahout.cf.taste.impl.common.LongPrimitiveIterator;
import org.apache.mahout.cf.taste.impl.recommender.GenericRecommendedItem;
import org.apache.mahout.cf.taste.model.DataModel;
import org.apache.mahout.cf.taste.model.PreferenceArray;
import org.apache.mahout.cf.taste.recommender.RecommendedItem;
import org.apache.mahout.cf.taste.similarity.PreferenceInferrer;
import org.apache.mahout.cf.taste.similarity.UserSimilarity;

public final class CosineCMGpu extends AbstractItemSimilarity implements UserSimilarity {

  static {
    System.loadLibrary("mahout_cms_jni");  // links libmahout_cms.so
  }

  // status codes of include/mahout_cms.h
  static final int CMS_E_PARAM = 1;
  static final int CMS_E_SHAPE = 2;
  static final int CMS_E_NO_SUCH_ID = 3;

  private final int depth;
  private final int width;
  private final CountMinSketchConfig config;  // per-owner shapes from the caller's config, or null
  private final double q;                     // per-owner shapes searched on the GPU (NaN: not used)
  private final long seed;
  private final boolean weighted;
  private final int device;
  // the DataModel as built (sorted owner IDs, offsets, item IDs in
  // getPreferencesFromUser order): recommendAll's getAllOtherItems source
  private volatile long[][] modelCsr;
  private final long[] hashA;  // a HashFunctionBuilder's drawn (a_i, b_i), or null: drawn from seed
  private final long[] hashB;
  private volatile long handle;  // cms_handle*
  /**
   * Every native call on the handle holds the read side; build() swaps in a
   * new table and close() ends it under the write side, so a handle is
   * destroyed only once no call that read it is still inside the library.
   */
  private final ReentrantReadWriteLock handleLock = new ReentrantReadWriteLock();
  private volatile int builtUsers = -1;  // DataModel.getNumUsers() / getNumItems() the table was built from
  private volatile int builtItems = -1;

  /** Hash rows a per-owner handle carries (CMS_MAX_DEPTH of include/mahout_cms.h). */
  static final int MAX_DEPTH = 32;

  /**
   * @param hfBuilderSeed the seed a HashFunctionBuilder(seed) would be built with
   *        (HashFunctionBuilder.java:23); the same seed gives the same buckets
   */
  public CosineCMGpu(DataModel dataModel, int depth, int width, long hfBuilderSeed, Weighting weighting, int device)
      throws TasteException {
    super(dataModel);
    if (!dataModel.hasPreferenceValues()) {  // CosineCM.java:38
      throw new IllegalArgumentException("DataModel doesn't have preference values");
    }
    this.depth = depth;
    this.width = width;
    this.config = null;
    this.q = Double.NaN;
    this.seed = hfBuilderSeed;
    this.weighted = weighting == Weighting.WEIGHTED;
    this.device = device;
    this.hashA = null;
    this.hashB = null;
    build();
  }

  /**
   * The reference's CosineCM(dataModel, weighting, conf, hfBuilder) (CosineCM.java:33-39):
   * each owner's sketch is sized by conf.getDelta/getEpsilon (the caller has run
   * conf.configure(dataModel, name) as before, or loaded its ser/ cache).
   */
  public CosineCMGpu(DataModel dataModel, Weighting weighting, CountMinSketchConfig conf, long hfBuilderSeed,
                     int device) throws TasteException {
    super(dataModel);
    if (!dataModel.hasPreferenceValues()) {  // CosineCM.java:38
      throw new IllegalArgumentException("DataModel doesn't have preference values");
    }
    this.depth = 0;
    this.width = 0;
    this.config = conf;
    this.q = Double.NaN;
    this.seed = hfBuilderSeed;
    this.weighted = weighting == Weighting.WEIGHTED;
    this.device = device;
    this.hashA = null;
    this.hashB = null;
    build();
  }

  /**
   * Per-owner shapes with CountMinSketchConfig(q)'s Fmeasure search
   * (CountMinSketchConfig.java:120-158) run on the GPU instead of the JVM.
   */
  public CosineCMGpu(DataModel dataModel, Weighting weighting, double q, long hfBuilderSeed, int device)
      throws TasteException {
    super(dataModel);
    if (!dataModel.hasPreferenceValues()) {  // CosineCM.java:38
      throw new IllegalArgumentException("DataModel doesn't have preference values");
    }
    this.depth = 0;
    this.width = 0;
    this.config = null;
    this.q = q;
    this.seed = hfBuilderSeed;
    this.weighted = weighting == Weighting.WEIGHTED;
    this.device = device;
    this.hashA = null;
    this.hashB = null;
    build();
  }

  /**
   * Per-owner shapes from the caller's config, hashing with parameters a
   * HashFunctionBuilder has drawn (HashFunctionParams.draw(builder, MAX_DEPTH)):
   * the backing of the same-package CosineCM replacement, whose constructors
   * take the builder itself (CosineCM.java:26-39).
   */
  CosineCMGpu(DataModel dataModel, Weighting weighting, CountMinSketchConfig conf, long[] hashA, long[] hashB,
              int device) throws TasteException {
    super(dataModel);
    if (!dataModel.hasPreferenceValues()) {  // CosineCM.java:38
      throw new IllegalArgumentException("DataModel doesn't have preference values");
    }
    if (hashA.length != MAX_DEPTH || hashB.length != MAX_DEPTH) {
      throw new IllegalArgumentException("one (a, b) pair per hash row: " + MAX_DEPTH);
    }
    this.depth = 0;
    this.width = 0;
    this.config = conf;
    this.q = Double.NaN;
    this.seed = 0L;
    this.weighted = weighting == Weighting.WEIGHTED;
    this.device = device;
    this.hashA = hashA.clone();
    this.hashB = hashB.clone();
    build();
  }

  private boolean perOwner() {
    return config != null || !Double.isNaN(q);
  }

  public CosineCMGpu(DataModel dataModel, int depth, int width, long hfBuilderSeed) throws TasteException {
    this(dataModel, depth, width, hfBuilderSeed, Weighting.UNWEIGHTED, -1);
  }

  /** DataModel -> CSR (sorted owner IDs, per-owner PreferenceArray order) -> GPU table. */
  private void build() throws TasteException {
    DataModel model = getDataModel();
    int n = model.getNumUsers();
    int numItems = model.getNumItems();
    long[] ids = new long[n];
    long[] offsets = new long[n + 1];
    int r = 0;
    long total = 0;
    LongPrimitiveIterator it = model.getUserIDs();
    while (it.hasNext()) {
      long id = it.nextLong();
      ids[r] = id;
      total += model.getPreferencesFromUser(id).length();
      offsets[++r] = total;
    }
    long[] keys = new long[(int) total];
    float[] vals = new float[(int) total];
    for (int i = 0; i < n; i++) {
      PreferenceArray prefs = model.getPreferencesFromUser(ids[i]);
      int base = (int) offsets[i];
      for (int j = 0; j < prefs.length(); j++) {
        keys[base + j] = prefs.getItemID(j);
        vals[base + j] = prefs.getValue(j);
      }
    }
    int fracBits = counterUnits(offsets, vals);
    modelCsr = new long[][] {ids, offsets, keys};
    long h = perOwner() ? nativeCreatePerOwner(seed, n, weighted, device, fracBits)
                        : nativeCreate(depth, width, seed, n, weighted, device, fracBits);
    try {
      if (hashA != null) {
        nativeSetHashParams(h, hashA, hashB);
      }
      nativeSetOwnerIds(h, ids);
      nativeIngestCsr(h, offsets, keys, vals);
      if (config != null) {
        double[] delta = new double[n];
        double[] epsilon = new double[n];
        for (int i = 0; i < n; i++) {
          delta[i] = config.getDelta(ids[i]);
          epsilon[i] = config.getEpsilon(ids[i]);
        }
        nativeSetOwnerDeltaEpsilon(h, delta, epsilon);
      } else if (perOwner()) {
        nativeConfigureOwnerShapes(h, q, model.getNumItems());
      }
      nativeFinalize(h);
    } catch (TasteException | RuntimeException e) {
      nativeDestroy(h);
      throw e;
    }
    handleLock.writeLock().lock();
    try {
      long old = handle;
      handle = h;
      builtUsers = n;
      builtItems = numItems;
      if (old != 0) {
        nativeDestroy(old);
      }
    } finally {
      handleLock.writeLock().unlock();
    }
  }

  /** The current handle, with the read side held: pair with release(). */
  private long acquire() throws TasteException {
    handleLock.readLock().lock();
    long h = handle;
    if (h == 0) {
      handleLock.readLock().unlock();
      throw new TasteException("CosineCMGpu is closed");
    }
    return h;
  }

  private void release() {
    handleLock.readLock().unlock();
  }

  /** The DataModel's user or item count differs from the one the table was built from. */
  boolean isStale() throws TasteException {
    DataModel model = getDataModel();
    return model.getNumUsers() != builtUsers || model.getNumItems() != builtItems;
  }

  /** Rebuild the device table from the DataModel as it is now. */
  void rebuild() throws TasteException {
    build();
  }

  /**
   * Counter representation for this DataModel.  Returns the smallest s with
   * every preference * 2^s an integer (1 for half-star ratings) when exact u32
   * counters in units of 2^-s can hold every owner's total (mass * 2^s < 2^32):
   * every similarity is then bit-identical and fast.  Otherwise -- negative,
   * non-finite or non-dyadic preferences, or masses past 2^32 units -- returns
   * -1: DoubleCountMinSketch's own fp64 counters (CMS_COUNTER_F64), which add
   * the preferences in DataModel order exactly as the reference does.
   */
  static int counterUnits(long[] offsets, float[] vals) {
    int s;
    try {
      s = fracBits(vals);
    } catch (TasteException e) {
      return -1;
    }
    for (float v : vals) {
      if (v < 0.0f || Float.isNaN(v) || Float.isInfinite(v)) {
        return -1;
      }
    }
    for (int r = 0; r + 1 < offsets.length; r++) {
      double mass = 0.0;
      for (long i = offsets[r]; i < offsets[r + 1]; i++) {
        mass += Math.scalb((double) vals[(int) i], s);
      }
      if (mass >= 4294967296.0) {
        return -1;
      }
    }
    return s;
  }

  /**
   * Smallest s with every preference * 2^s an integer (1 for half-star
   * ratings): the library keeps counters in units of 2^-s, which leaves every
   * similarity bit-identical and point queries in preference units.
   */
  static int fracBits(float[] vals) throws TasteException {
    int s = 0;
    for (float v : vals) {
      if (v == 0.0f || Float.isNaN(v) || Float.isInfinite(v)) {
        continue;  // counterUnits() sends non-finite values to the fp64 counters
      }
      int bits = Float.floatToIntBits(Math.abs(v));
      int exp = ((bits >>> 23) & 0xff) - 150;  // v = mant * 2^exp with a 24-bit mant
      int mant = (bits & 0x7fffff) | (((bits >>> 23) & 0xff) == 0 ? 0 : 0x800000);
      if (((bits >>> 23) & 0xff) == 0) {
        exp = -149;
      }
      exp += Integer.numberOfTrailingZeros(mant);
      s = Math.max(s, -exp);
    }
    if (s > 31) {
      throw new TasteException("preference values need more than 31 fractional bits");
    }
    return s;
  }

  /** CosineCM.userSimilarity (CosineCM.java:83-96). */
  @Override
  public double userSimilarity(long userID1, long userID2) throws TasteException {
    long h = acquire();
    try {
      return nativeSimilarity(h, userID1, userID2, false);
    } finally {
      release();
    }
  }

  @Override
  public void setPreferenceInferrer(PreferenceInferrer inferrer) {
    if (inferrer == null) {
      throw new IllegalArgumentException("inferrer is null");
    }
    // the sketch cosine does not infer preferences (as CosineCM)
  }

  /** Sketch cosine between owners; owners are items over a transposed DataModel. */
  @Override
  public double itemSimilarity(long itemID1, long itemID2) throws TasteException {
    long h = acquire();
    try {
      return nativeSimilarity(h, itemID1, itemID2, true);
    } finally {
      release();
    }
  }

  @Override
  public double[] itemSimilarities(long itemID1, long[] itemID2s) throws TasteException {
    long h = acquire();
    try {
      return nativeSimilarities(h, itemID1, itemID2s);
    } finally {
      release();
    }
  }

  /** GenericUserBasedRecommender.mostSimilarUserIDs + TopItems.getTopUsers semantics. */
  public long[] mostSimilarIDs(long ownerID, int howMany) throws TasteException {
    if (howMany < 1) {
      throw new IllegalArgumentException("howMany must be at least 1");
    }
    long h = acquire();
    try {
      return nativeMostSimilar(h, ownerID, howMany);
    } finally {
      release();
    }
  }

  /** DoubleCountMinSketch.get(key) on the owner's sketch (point query). */
  public double pointQuery(long ownerID, long key) throws TasteException {
    long h = acquire();
    try {
      return nativePointQuery(h, ownerID, key);
    } finally {
      release();
    }
  }

  /** {width, depth} of the owner's own sketch (per-owner shapes). */
  int[] ownerShape(long ownerID) throws TasteException {
    long h = acquire();
    try {
      return nativeOwnerShape(h, ownerID);
    } finally {
      release();
    }
  }

  /** The owner's own sketch, [depth][width] row-major as DoubleCountMinSketch stores it. */
  double[] readOwnerSketch(long ownerID) throws TasteException {
    long h = acquire();
    try {
      return nativeReadOwnerSketch(h, ownerID);
    } finally {
      release();
    }
  }

  /**
   * GenericUserBasedRecommender.doEstimatePreference(user, neighborhood, item)
   * with the CosineCM point query, for many items in one call; NaN where fewer
   * than two neighbours carry data. Pass capMin/capMax = NaN for no capper.
   */
  public float[] estimatePreferences(long userID, long[] neighborhood, long[] itemIDs, float capMin, float capMax)
      throws TasteException {
    long h = acquire();
    try {
      return nativeEstimatePreferences(h, userID, neighborhood, itemIDs, capMin, capMax);
    } finally {
      release();
    }
  }

  /**
   * GenericUserBasedRecommender.recommend(userID, howMany) (:84-105) with
   * NearestNUserNeighborhood(neighborhoodSize) for every user of userIDs in
   * one call (cms_recommend_batch): the neighbourhoods from one all-owners
   * top-n pass, the candidates in FastIDSet iteration order and
   * TopItems.getTopItems (JDK PriorityQueue tie order) in the library, every
   * estimate in one device batch. Pass capMin/capMax = NaN for no capper.
   * Element u is user u's list, equal to recommend(userIDs[u], howMany).
   */
  public List<List<RecommendedItem>> recommendAll(long[] userIDs, int neighborhoodSize, int howMany,
                                                  boolean includeKnownItems, float capMin, float capMax)
      throws TasteException {
    long h = acquire();
    try {
      long[][] csr = modelCsr;
      long[][] lists = nativeTopKAll(h, neighborhoodSize);  // rows in ascending owner-ID order
      long[] nbOffsets = new long[userIDs.length + 1];
      for (int u = 0; u < userIDs.length; u++) {
        int r = java.util.Arrays.binarySearch(csr[0], userIDs[u]);
        if (r < 0) {
          throw new NoSuchUserException(userIDs[u]);
        }
        nbOffsets[u + 1] = nbOffsets[u] + lists[r].length;
      }
      long[] nbIds = new long[(int) nbOffsets[userIDs.length]];
      for (int u = 0; u < userIDs.length; u++) {
        long[] nb = lists[java.util.Arrays.binarySearch(csr[0], userIDs[u])];
        System.arraycopy(nb, 0, nbIds, (int) nbOffsets[u], nb.length);
      }
      int[] counts = new int[userIDs.length];
      long[] items = new long[userIDs.length * howMany];
      float[] values = new float[userIDs.length * howMany];
      nativeRecommendBatch(h, userIDs, nbOffsets, nbIds, csr[0], csr[1], csr[2], howMany, includeKnownItems, capMin,
                           capMax, counts, items, values);
      List<List<RecommendedItem>> out = new ArrayList<>(userIDs.length);
      for (int u = 0; u < userIDs.length; u++) {
        List<RecommendedItem> l = new ArrayList<>(counts[u]);
        for (int j = 0; j < counts[u]; j++) {
          l.add(new GenericRecommendedItem(items[u * howMany + j], values[u * howMany + j]));
        }
        out.add(l);
      }
      return out;
    } finally {
      release();
    }
  }

  /**
   * mostSimilarIDs for every owner at once (each unordered pair computed once):
   * row r of the result holds the IDs for the r-th owner in ascending ID order.
   */
  public long[][] allMostSimilarIDs(int howMany) throws TasteException {
    long h = acquire();
    try {
      return nativeTopKAll(h, howMany);
    } finally {
      release();
    }
  }

  /**
   * The same lists after streaming COO batches (cms_top_k_refresh): only the
   * pairs of owners touched since the previous call are recomputed. This
   * class re-ingests its DataModel as CSR on refresh(), which makes the next
   * call a whole job; the incremental path serves streaming callers.
   */
  public long[][] allMostSimilarIDsRefreshed(int howMany) throws TasteException {
    long h = acquire();
    try {
      return nativeTopKRefresh(h, howMany);
    } finally {
      release();
    }
  }

  @Override
  public void refresh(Collection<Refreshable> alreadyRefreshed) {
    super.refresh(alreadyRefreshed);
    try {
      build();
    } catch (TasteException te) {
      throw new IllegalStateException(te);
    }
  }

  public void close() {
    handleLock.writeLock().lock();
    try {
      if (handle != 0) {
        nativeDestroy(handle);
        handle = 0;
      }
    } finally {
      handleLock.writeLock().unlock();
    }
  }

  @Override
  public String toString() {
    return "CosineCMGpu[dataModel:" + getDataModel()
        + (perOwner() ? ",per-owner shapes" : ",d:" + depth + ",w:" + width) + ']';
  }

  // --- JNI (integration/jni/mahout_cms_jni.c) --------------------------------
  private static native long nativeCreate(int depth, int width, long seed, long numOwners, boolean weighted,
                                          int device, int fracBits) throws TasteException;
  private static native long nativeCreatePerOwner(long seed, long numOwners, boolean weighted, int device,
                                                  int fracBits) throws TasteException;
  private static native void nativeConfigureOwnerShapes(long h, double q, long numKeys) throws TasteException;
  private static native void nativeSetOwnerDeltaEpsilon(long h, double[] delta, double[] epsilon)
      throws TasteException;
  private static native void nativeSetOwnerIds(long h, long[] ids) throws TasteException;
  private static native void nativeSetHashParams(long h, long[] a, long[] b) throws TasteException;
  private static native int[] nativeOwnerShape(long h, long id) throws TasteException;
  private static native double[] nativeReadOwnerSketch(long h, long id) throws TasteException;
  private static native void nativeIngestCsr(long h, long[] offsets, long[] keys, float[] vals) throws TasteException;
  private static native void nativeFinalize(long h) throws TasteException;
  private static native double nativeSimilarity(long h, long id1, long id2, boolean itemIds) throws TasteException;
  private static native double[] nativeSimilarities(long h, long id1, long[] ids2) throws TasteException;
  private static native long[] nativeMostSimilar(long h, long id, int k) throws TasteException;
  private static native double nativePointQuery(long h, long id, long key) throws TasteException;
  private static native float[] nativeEstimatePreferences(long h, long user, long[] neighbors, long[] items,
                                                          float capMin, float capMax) throws TasteException;
  private static native long[][] nativeTopKAll(long h, int k) throws TasteException;
  private static native void nativeRecommendBatch(long h, long[] users, long[] nbOffsets, long[] nbIds, long[] modelIds,
                                                  long[] prefOffsets, long[] prefItems, int howMany,
                                                  boolean includeKnown, float capMin, float capMax, int[] outCounts,
                                                  long[] outItems, float[] outValues) throws TasteException;
  private static native long[][] nativeTopKRefresh(long h, int k) throws TasteException;
  private static native void nativeDestroy(long h);
}
