/*
 * Same-package, same-name replacement of the reference's
 * org.apache.mahout.cf.taste.impl.similarity.CosineCM
 * (mr/src/main/java/org/apache/mahout/cf/taste/impl/similarity/CosineCM.java),
 * backed by libmahout_cms.so through CosineCMGpu and the JNI shim.
 *
 * Why a replacement class: GenericUserBasedRecommender.doEstimatePreference
 * tests `similarity instanceof CosineCM` and then calls
 * `sim.getExportedCMProfile(userID).get(itemID)` for the sketch point query
 * (GenericUserBasedRecommender.java:139-159), and CosineCM is final
 * (CosineCM.java:17).  Put this class's jar ahead of mahout-mr on the
 * classpath (or drop the reference's class file) and every caller --
 * recommenders, evaluators, Refreshable chains -- runs unchanged on the GPU.
 *
 * Contract kept from the reference:
 *  - constructors (DataModel, CountMinSketchConfig, HashFunctionBuilder) and
 *    (DataModel, Weighting, CountMinSketchConfig, HashFunctionBuilder)
 *    (CosineCM.java:26-39), IllegalArgumentException without preference values;
 *  - userSimilarity(u1, u2): u1's sketch at u2's (delta, epsilon) against u2's
 *    own sketch, min-over-rows cosine, normalizeWeightResult(r, 1, 0)
 *    (CosineCM.java:83-96) -- bit-identical; NoSuchUserException for an
 *    unknown ID, TasteException for an owner the config cannot shape (the
 *    CMException of exportProfile, :45-46);
 *  - getExportedCMProfile(id): a DoubleCountMinSketch with the owner's own
 *    shape and counters (:60-67), cached per ID as the reference caches it;
 *    its get(key) -- the recommender's point query -- is answered by the GPU
 *    (cms_point_query, the same fp64 value);
 *  - everything else (itemSimilarity as AbstractSimilarity's exact co-rated
 *    cosine, computeResult) is as before; refresh(Collection) and toString()
 *    are AbstractSimilarity's own: both are final there
 *    (AbstractSimilarity.java:333,339), so this class cannot override them.
 *
 * Refresh semantics.  AbstractSimilarity.refresh refreshes the DataModel and
 * re-reads its getNumUsers()/getNumItems() (AbstractSimilarity.java:53-62).
 * The reference's CosineCM keeps its `sketches` cache across a refresh (it is
 * never cleared, CosineCM.java:60-67) and rebuilds u1's sketch on every
 * userSimilarity call.  Here both sketches live on the device, so every entry
 * point first compares the DataModel's user and item counts with the ones the
 * device table was built from and, when they differ (a refreshed model that
 * gained or lost users or items), rebuilds the table and drops the cached
 * profiles.  A refresh that only changes preference values keeps the counts:
 * call rebuild() after it (the reference would serve such a change for u1
 * but not for its cached u2 sketches).
 * The hash functions are the caller's own HashFunctionBuilder: its drawn
 * (a_i, b_i) are installed on the device (HashFunctionParams.draw,
 * cms_set_hash_params), so even a clock-seeded builder hashes identically.
 *
 * NOTE: not compiled in this image (no JDK); tests/test_gpu_cosinecm_dropin.py
 * replays this class's C-ABI call sequence through ctypes against the oracle.
 */
package org.apache.mahout.cf.taste.impl.similarity;

import java.util.concurrent.ConcurrentHashMap;
import java.lang.reflect.Field;

import org.apache.mahout.cf.taste.common.TasteException;
import org.apache.mahout.cf.taste.common.Weighting;
import org.apache.mahout.cf.taste.impl.common.AbstractCountMinSketch;
import org.apache.mahout.cf.taste.impl.common.CountMinSketchConfig;
import org.apache.mahout.cf.taste.impl.common.DoubleCountMinSketch;
import org.apache.mahout.cf.taste.impl.common.HashFunctionBuilder;
import org.apache.mahout.cf.taste.impl.common.HashFunctionParams;
import org.apache.mahout.cf.taste.model.DataModel;

import com.google.common.base.Preconditions;

import gnu.trove.list.array.TDoubleArrayList;

public final class CosineCM extends AbstractSimilarity {

  private final HashFunctionBuilder hfBuilder;
  private final CountMinSketchConfig config;
  private final ConcurrentHashMap<Long, DoubleCountMinSketch> sketches;
  private final CosineCMGpu gpu;

  /**
   * @throws IllegalArgumentException if {@link DataModel} does not have preference values
   */
  public CosineCM(DataModel dataModel, CountMinSketchConfig conf, HashFunctionBuilder hfBuilder_)
      throws TasteException {
    this(dataModel, Weighting.UNWEIGHTED, conf, hfBuilder_);
  }

  /**
   * @throws IllegalArgumentException if {@link DataModel} does not have preference values
   */
  public CosineCM(DataModel dataModel, Weighting weighting, CountMinSketchConfig conf,
                  HashFunctionBuilder hfBuilder_) throws TasteException {
    super(dataModel, weighting, false);
    Preconditions.checkArgument(dataModel.hasPreferenceValues(), "DataModel doesn't have preference values");
    config = conf;
    hfBuilder = hfBuilder_;
    sketches = new ConcurrentHashMap<Long, DoubleCountMinSketch>(Math.max(16, dataModel.getNumUsers()));
    long[][] ab = HashFunctionParams.draw(hfBuilder_, CosineCMGpu.MAX_DEPTH);
    gpu = new CosineCMGpu(dataModel, weighting, conf, ab[0], ab[1], -1);
  }

  /**
   * The owner's own sketch (CosineCM.java:60-67): shape from the config's
   * (delta, epsilon), counters read from the device once and cached.
   */
  public DoubleCountMinSketch getExportedCMProfile(long userID) throws TasteException {
    ensureCurrent();
    DoubleCountMinSketch cm = sketches.get(userID);
    if (cm == null) {
      int[] shape = gpu.ownerShape(userID);  // NoSuchUserException / TasteException as exportProfile
      double[] counters = gpu.readOwnerSketch(userID);
      try {
        cm = new DeviceSketch(shape[0], shape[1], hfBuilder, gpu, userID, counters);
      } catch (AbstractCountMinSketch.CMException ex) {
        throw new TasteException("CountMinSketch error:" + ex.getMessage());
      }
      DoubleCountMinSketch prev = sketches.putIfAbsent(userID, cm);
      if (prev != null) {
        cm = prev;
      }
    }
    return cm;
  }

  @Override
  double computeResult(int n, double sumXY, double sumX2, double sumY2, double sumXYdiff2) {
    if (n == 0) {
      return Double.NaN;
    }
    double denominator = Math.sqrt(sumX2) * Math.sqrt(sumY2);
    if (denominator == 0.0) {
      return Double.NaN;
    }
    return sumXY / denominator;
  }

  /** CosineCM.userSimilarity (CosineCM.java:83-96) as one cms_similarity call. */
  @Override
  public double userSimilarity(long userID1, long userID2) throws TasteException {
    ensureCurrent();
    return gpu.userSimilarity(userID1, userID2);
  }

  /**
   * Rebuild the device table from the DataModel as it is now and drop the
   * cached profiles (after a refresh that changed preference values but not
   * the user or item counts).
   */
  public void rebuild() throws TasteException {
    synchronized (gpu) {
      gpu.rebuild();
      sketches.clear();
    }
  }

  /** Lazy refresh: the DataModel gained or lost users or items since the build. */
  private void ensureCurrent() throws TasteException {
    if (gpu.isStale()) {
      synchronized (gpu) {
        if (gpu.isStale()) {
          gpu.rebuild();
          sketches.clear();
        }
      }
    }
  }

  /**
   * getExportedCMProfile's result: a DoubleCountMinSketch holding the owner's
   * counters (so toString and DoubleCountMinSketch.cosine see the reference's
   * values) whose point query get(key) runs on the GPU.  Read-only: the
   * reference's cached profile could be mutated by a caller, but the GPU table
   * is the similarity's source of truth here, so update() refuses.
   */
  static final class DeviceSketch extends DoubleCountMinSketch {
    private final CosineCMGpu gpu;
    private final long owner;

    DeviceSketch(int width, int depth, HashFunctionBuilder hfb, CosineCMGpu gpu, long owner, double[] counters)
        throws AbstractCountMinSketch.CMException {
      super(width, depth, hfb);
      this.gpu = gpu;
      this.owner = owner;
      TDoubleArrayList count = countList(this);
      for (int i = 0; i < counters.length; i++) {
        count.set(i, counters[i]);
      }
    }

    private static TDoubleArrayList countList(DoubleCountMinSketch sk) {
      try {
        Field f = DoubleCountMinSketch.class.getDeclaredField("count");
        f.setAccessible(true);
        return (TDoubleArrayList) f.get(sk);
      } catch (NoSuchFieldException | IllegalAccessException e) {
        throw new IllegalStateException("DoubleCountMinSketch.count not writable", e);
      }
    }

    /** DoubleCountMinSketch.get(key) (DoubleCountMinSketch.java:94-103) via cms_point_query. */
    @Override
    public double get(long key) {
      try {
        return gpu.pointQuery(owner, key);
      } catch (TasteException e) {
        throw new IllegalStateException(e);
      }
    }

    @Override
    public void update(long key, double increment) {
      throw new UnsupportedOperationException("GPU-backed sketch profile is read-only");
    }
  }
}
