"""Pure-Python restatement of the JDK/BigInteger semantics the reference hash
relies on.  TEST INFRASTRUCTURE ONLY: an independent second restatement used to
cross-check the C oracle (oracle/cms_oracle.c) on hash parameters and indices.

Python integers are arbitrary precision and ``%`` with a positive modulus is
non-negative, exactly ``java.math.BigInteger.mod`` -- so ``hash`` below is a
line-for-line statement of T/impl/common/HashFunction.java:31-34 with no
128-bit tricks, which is what makes it a useful independent check.

T/ = mr/src/main/java/org/apache/mahout/cf/taste/ under the reference.
"""

MULT = 0x5DEECE66D
ADD = 0xB
MASK = (1 << 48) - 1
PRIME = 9223372036854775783  # T/impl/common/HashFunctionBuilder.java:24 (2^63 - 25)


def _to_int(v: int, bits: int) -> int:
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


class JavaRandom:
    """java.util.Random (JDK published algorithm)."""

    def __init__(self, seed: int):
        self.seed = (seed ^ MULT) & MASK

    def next(self, bits: int) -> int:
        self.seed = (self.seed * MULT + ADD) & MASK
        return _to_int(self.seed >> (48 - bits), 32)

    def next_int(self) -> int:
        return self.next(32)

    def next_long(self) -> int:
        return _to_int((self.next(32) << 32) + self.next(32), 64)


def java_abs_long(v: int) -> int:
    """Math.abs(long): Long.MIN_VALUE stays negative."""
    return _to_int(-v, 64) if v < 0 else v


def hash_params(seed: int, depth: int):
    """HashFunctionBuilder(seed).getHashFunction(i, w) params, i < depth
    (T/impl/common/HashFunctionBuilder.java:23-29, 42-56)."""
    r = JavaRandom(seed)
    a, b = [], []
    for _ in range(depth):
        a.append(java_abs_long(r.next_long()))
        b.append(java_abs_long(r.next_long()))
    return a, b


def hash_(a: int, b: int, width: int, key: int) -> int:
    """HashFunction.hash: a*k + b mod p mod w in big integers."""
    return ((a * key + b) % PRIME) % width
