/*
 * Reads the (a_i, b_i) a HashFunctionBuilder has drawn, so the GPU sketches
 * (libmahout_cms.so, cms_set_hash_params) hash with exactly the builder the
 * caller handed to CosineCM -- including `new HashFunctionBuilder()`, whose
 * seed is the clock and cannot be recovered.
 *
 * Lives in the reference's package org.apache.mahout.cf.taste.impl.common
 * because HashFunctionBuilder.getHashFunction(i, size) is package-private
 * (HashFunctionBuilder.java:40-61).  Asking for rows 0..count-1 draws their
 * parameters in row order exactly as the reference's lazy draw would (row i's
 * pair never depends on the size argument or on when it is drawn), so the
 * builder stays usable by other sketches afterwards.  The drawn lists are
 * private fields (randomParamA / randomParamB, TLongArrayList), read by
 * reflection under the builder's own lock.
 *
 * NOTE: not compiled in this image (no JDK); see INTEGRATION.md.
 */
package org.apache.mahout.cf.taste.impl.common;

import java.lang.reflect.Field;

import gnu.trove.list.array.TLongArrayList;

public final class HashFunctionParams {

  private HashFunctionParams() {
  }

  /** {a[0..count), b[0..count)} of the builder's first count hash functions. */
  public static long[][] draw(HashFunctionBuilder builder, int count) {
    if (count < 1) {
      throw new IllegalArgumentException("count must be at least 1");
    }
    long[] a = new long[count];
    long[] b = new long[count];
    synchronized (builder) {  // getHashFunction's draw block locks the builder too
      builder.getHashFunction(count - 1, 1);  // draws rows 0..count-1 if not drawn yet
      TLongArrayList pa = field(builder, "randomParamA");
      TLongArrayList pb = field(builder, "randomParamB");
      for (int i = 0; i < count; i++) {
        a[i] = pa.get(i);
        b[i] = pb.get(i);
      }
    }
    return new long[][] {a, b};
  }

  private static TLongArrayList field(HashFunctionBuilder builder, String name) {
    try {
      Field f = HashFunctionBuilder.class.getDeclaredField(name);
      f.setAccessible(true);
      return (TLongArrayList) f.get(builder);
    } catch (NoSuchFieldException | IllegalAccessException e) {
      throw new IllegalStateException("HashFunctionBuilder." + name + " not readable", e);
    }
  }
}
