"""CPU oracle: pure-Python restatement of the reference's LDE / NTT / Merkle / FRI-commit path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the
checker.  The product path (`zk-stark-tutor_amd/`) never imports it.

Every function restates the algorithm of the reference crate
(SpekalsG3/zk-stark-tutor, Rust) at the cited `file:line` under
`/root/reference/src/`.  The two third-party hashes the reference pulls from
crates that are not vendored (`blake2 0.10.6` -> BLAKE2b-512, RFC 7693;
`sha3 0.10.8` -> SHAKE256, FIPS 202) are taken from Python's `hashlib`, which
implements the same published algorithms.  Parity of this restatement is
pinned by the reference's own known-answer tests, transcribed into
`tests/golden/reference_kats.json` and checked by `tests/test_oracle_kats.py`.

Field elements are Python ints in canonical form [0, p).
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence, Tuple

# field/field.rs:10  FIELD_PRIME = 1 + 407 * 2^119
P = 1 + 407 * (1 << 119)
# field/field.rs:41-44  Field::generator()
GENERATOR = 85408008396924667383611388730472331217
# crypto/shake256.rs:5
PROOF_BYTES = 32


# ---------------------------------------------------------------- field (L1)

def sub_mod(a: int, b: int) -> int:
    """field/field.rs:101-107 (3-way compare)."""
    if a > b:
        return a - b
    if a == b:
        return 0
    return P - b + a


def add_mod(a: int, b: int) -> int:
    """field/field.rs:109-115: a + b == sub_mod(a, p - b); b == 0 returns a."""
    if b == 0:
        return a
    return sub_mod(a, P - b)


def neg_mod(a: int) -> int:
    """field/field.rs:151-157."""
    return 0 if a == 0 else P - a


def mul_mod(a: int, b: int) -> int:
    """field/field.rs:117-131 (bit-serial double-and-add; exact product mod p)."""
    return (a * b) % P


def u_xgcd(a: int, b: int) -> Tuple[int, int, int]:
    """utils/xgcd.rs:22-48 (unsigned-input extended Euclid, Hurchalla form)."""
    x1, y1 = 1, 0
    x0, y0 = 0, 1
    r0, r1 = a, b
    q = 0
    while r1 != 0:
        x2 = x0 - q * x1
        y2 = y0 - q * y1
        x0, y0 = x1, y1
        x1, y1 = x2, y2
        q = r0 // r1
        r0, r1 = r1, r0 - q * r1
    return x1, y1, r0


def inv(a: int) -> int:
    """field/field.rs:160-169: inverse via u_xgcd; inv(0) == 0 (xgcd yields 0)."""
    s, _, _ = u_xgcd(a, P)
    if s > 0:
        return s
    if s == 0:
        return 0
    return sub_mod(P, -s)


def div(a: int, b: int) -> int:
    """field/field_element.rs:82-90: asserts b != 0, then a * b^-1."""
    if b == 0:
        raise ZeroDivisionError("divide by zero")
    return mul_mod(a, inv(b))


def fpow(x: int, e: int) -> int:
    """field/field_element.rs:108-143: left-to-right square-and-multiply over bitlen(e).

    The loop computes x^e mod p (x^0 = 1, including 0^0); CPython's three-argument pow
    returns the same value and is used for speed."""
    return pow(x, e, P)


def primitive_nth_root(n: int) -> int:
    """field/field.rs:58-71: square the generator down from order 2^119."""
    assert n & (n - 1) == 0 and n <= (1 << 119), "n must be a power of two <= 2^119"
    root = GENERATOR
    order = 1 << 119
    while order != n:
        root = fpow(root, 2)
        order //= 2
    return root


def sample(data: bytes) -> int:
    """field/field.rs:87-99: fold (acc << 8) ^ b over u128 (= last 16 bytes BE), mod p."""
    acc = 0
    for b in data:
        acc = ((acc << 8) ^ b) & ((1 << 128) - 1)
    return acc % P


def fe_to_leaf_bytes(v: int) -> bytes:
    """field/field_element.rs:46-50: Into<Bytes> is the decimal ASCII string of the value."""
    return str(v).encode("ascii")


# ------------------------------------------------------------- transforms (L2)

def bit_reverse_copy(inputs: Sequence[int]) -> List[int]:
    """utils/bit_reverse_copy.rs:3-34: zero-pad to next_pow2, x[k] -> position rev(k)."""
    if len(inputs) < 2:
        return list(inputs)
    n = 1 << (len(inputs) - 1).bit_length()
    padded = list(inputs) + [0] * (n - len(inputs))
    logn = n.bit_length() - 1
    out = [0] * n
    for k, el in enumerate(padded):
        out[int(format(k, "0%db" % logn)[::-1], 2)] = el
    return out


def ntt(root: int, inputs: Sequence[int]) -> List[int]:
    """fft/ntt.rs:7-49: bit_reverse_copy, powtable[k] = root^k (k < n/2), radix-2 DIT.

    The butterfly graph (and therefore the result, for ANY root) is the
    reference's: stage `size`, twiddle powtable[k * n/size], (e + w*o, e - w*o).
    """
    if len(inputs) == 0:
        raise IndexError("ntt of empty input (reference indexes inputs[0])")
    x = bit_reverse_copy(inputs)
    n = len(x)
    powtable = []
    t = 1
    for _ in range(n // 2):
        powtable.append(t)
        t = mul_mod(t, root)
    size = 1
    while size < n:
        size <<= 1
        half = size // 2
        step = n // size
        for i in range(0, n, size):
            k = 0
            for j in range(i, i + half):
                l = j + half
                e = x[j]
                o = mul_mod(x[l], powtable[k])
                x[j] = add_mod(e, o)
                x[l] = sub_mod(e, o)
                k += step
    return x


def intt(root: int, inputs: Sequence[int]) -> List[int]:
    """fft/ntt.rs:51-68: len < 2 returns the input; else ntt(root^-1) * n^-1."""
    if len(inputs) < 2:
        return list(inputs)
    n = 1 << (len(inputs) - 1).bit_length()
    ninv = inv(n)
    return [mul_mod(ninv, v) for v in ntt(inv(root), inputs)]


def scale(coeffs: Sequence[int], factor: int) -> List[int]:
    """field/polynomial.rs:109-121: c_i <- factor^i * c_i."""
    out = []
    pw = 1
    for c in coeffs:
        out.append(mul_mod(pw, c))
        pw = mul_mod(pw, factor)
    return out


def fast_coset_evaluate(generator: int, root_order: int, offset: int, coeffs: Sequence[int]) -> List[int]:
    """fft/ntt_arithmetics.rs:161-170 (the LDE): scale(offset), zero-pad to root_order, ntt(generator)."""
    if len(coeffs) > root_order:
        raise ValueError("polynomial longer than root_order (reference panics on usize underflow)")
    c = scale(coeffs, offset)
    c += [0] * (root_order - len(c))
    return ntt(generator, c)


def evaluate(coeffs: Sequence[int], x: int) -> int:
    """Horner evaluation (the algebraic cross-check used by fft/ntt.rs:98-104)."""
    acc = 0
    for c in reversed(coeffs):
        acc = add_mod(mul_mod(acc, x), c)
    return acc


# ---------------------------------------------------------------- hashes (L1)

def blake2b512(data: bytes) -> bytes:
    """crypto/blake2b512.rs:4-14 (crate blake2 0.10.6: unkeyed BLAKE2b, 64-byte digest)."""
    return hashlib.blake2b(data, digest_size=64).digest()


def shake256(data: bytes, num_bytes: int) -> bytes:
    """crypto/shake256.rs:7-19 (crate sha3 0.10.8: SHAKE256 XOF)."""
    return hashlib.shake_256(data).digest(num_bytes)


# ----------------------------------------------------------- Merkle tree (L3)

def merkle_leaf_digests(values: Sequence[int]) -> List[bytes]:
    """merkle_root.rs:25-30: leaf digest = blake2b512(decimal(value))."""
    return [blake2b512(fe_to_leaf_bytes(v)) for v in values]


def merkle_levels(values: Sequence[int]) -> List[List[bytes]]:
    """All levels of the tree commit_ (merkle_root.rs:7-19) builds.

    commit_ halves recursively over natural order, so a node is
    blake2b512(left || right) of adjacent pairs, bottom-up; a 1-element tree's
    root is the leaf digest.  levels[0] = leaf digests, levels[-1] = [root].
    """
    n = len(values)
    if n == 0 or n & (n - 1):
        raise ValueError("Leafs len must be power of two")
    level = merkle_leaf_digests(values)
    levels = [level]
    while len(level) > 1:
        level = [blake2b512(level[2 * i] + level[2 * i + 1]) for i in range(len(level) // 2)]
        levels.append(level)
    return levels


def merkle_commit(values: Sequence[int]) -> bytes:
    """merkle_root.rs:21-32 MerkleRoot::commit."""
    return merkle_levels(values)[-1][0]


def merkle_open(index: int, values: Sequence[int]) -> List[bytes]:
    """merkle_root.rs:34-66 MerkleRoot::open: sibling digests from leaf level up."""
    return merkle_open_levels(index, merkle_levels(values))


def merkle_open_levels(index: int, levels: List[List[bytes]]) -> List[bytes]:
    """merkle_open on precomputed levels (same output; avoids the reference's O(n) rehash per open)."""
    n = len(levels[0])
    if not 0 <= index < n:
        raise ValueError("cannot open invalid index")
    if n < 2:
        raise ValueError("cannot open a 1-leaf tree (reference indexes leafs[1 - index])")
    path = []
    idx = index
    for level in levels[:-1]:
        path.append(level[idx ^ 1])
        idx >>= 1
    return path


def merkle_verify(root: bytes, index: int, path: Sequence[bytes], value: int) -> bool:
    """merkle_root.rs:69-95 MerkleRoot::verify."""
    if not index < (1 << len(path)):
        raise ValueError("Cannot verify invalid index")
    h = blake2b512(fe_to_leaf_bytes(value))
    for sib in path:
        h = blake2b512(h + sib) if index % 2 == 0 else blake2b512(sib + h)
        index >>= 1
    return h == root


# -------------------------------------------------------- proof stream (L3)

# stark/proof_stream_enum.rs:8-15  (object code = enum discriminant)
ROOT, CODEWORD, PATH, LEAFS, VALUE = 0, 1, 2, 3, 4


def _u128be(v: int) -> bytes:
    return v.to_bytes(16, "big")


def object_payload(obj) -> Tuple[int, bytes, bool]:
    """stark/proof_stream_enum.rs:67-127 to_bytes: (code, payload, carries_field)."""
    code, val = obj
    if code == ROOT:
        return ROOT, bytes(val), False
    if code == CODEWORD:
        return CODEWORD, b"".join(_u128be(v) for v in val), len(val) > 0
    if code == PATH:
        return PATH, b"".join(len(b).to_bytes(8, "big") + bytes(b) for b in val), False
    if code == LEAFS:
        return LEAFS, b"".join(_u128be(v) for v in val), True
    if code == VALUE:
        return VALUE, _u128be(val), True
    raise ValueError("unknown object code")


def serialize(objects: Sequence) -> bytes:
    """stark/proof_stream_enum.rs:161-190 Digest for &[StarkProofStreamEnum].

    16-byte BE field order (0 when no object carries a field element), then per
    object [code u8][payload len u64 BE][payload].
    """
    body = []
    has_field = False
    for obj in objects:
        code, payload, f = object_payload(obj)
        has_field = has_field or f
        body.append(bytes([code]) + len(payload).to_bytes(8, "big") + payload)
    return _u128be(P if has_field else 0) + b"".join(body)


def deserialize(data: bytes) -> list:
    """stark/stark.rs:30-67 deser_independent_proof_stream + proof_stream_enum.rs:129-159 from_bytes:
    the objects of a serialized stream (the field order, when present, must be P)."""
    order = int.from_bytes(data[:16], "big")
    assert order in (0, P), "serialized field differs from Stark's field"
    pos, out = 16, []
    while pos < len(data):
        code = data[pos]
        size = int.from_bytes(data[pos + 1:pos + 9], "big")
        pl = data[pos + 9:pos + 9 + size]
        assert len(pl) == size, "truncated object"
        pos += 9 + size
        if code == ROOT:
            out.append((ROOT, bytes(pl)))
        elif code in (CODEWORD, LEAFS):
            vals = [int.from_bytes(pl[i:i + 16], "big") for i in range(0, size, 16)]
            out.append((code, vals if code == CODEWORD else tuple(vals)))
        elif code == PATH:
            path, q = [], 0
            while q < size:
                n = int.from_bytes(pl[q:q + 8], "big")
                path.append(bytes(pl[q + 8:q + 8 + n]))
                q += 8 + n
            out.append((PATH, path))
        elif code == VALUE:
            out.append((VALUE, int.from_bytes(pl, "big")))
        else:
            raise ValueError("unknown object code")
    return out


class IndependentProofStream:
    """proof_stream.rs:15-78 (the in-memory transcript)."""

    def __init__(self, objects=None):
        self.objects = list(objects or [])
        self.read_index = 0

    def digest(self) -> bytes:
        return serialize(self.objects)

    def fiat_shamir_prover(self, num_bytes: int) -> bytes:
        return shake256(self.digest(), num_bytes)

    def fiat_shamir_verifier(self, num_bytes: int) -> bytes:
        return shake256(serialize(self.objects[: self.read_index]), num_bytes)

    def push(self, obj) -> None:
        self.objects.append(obj)

    def pull(self):
        assert self.read_index < len(self.objects), "Cannot pull, queue is empty"
        obj = self.objects[self.read_index]
        self.read_index += 1
        return obj


class SignatureProofStream(IndependentProofStream):
    """rescue_prime/proof_stream.rs:9-61: Fiat-Shamir input prefixed by [len u64 BE][blake2b(doc)]."""

    def __init__(self, document: bytes, objects=None):
        super().__init__(objects)
        self.prefix = blake2b512(document)

    def _prefix(self) -> bytes:
        return len(self.prefix).to_bytes(8, "big") + self.prefix

    def fiat_shamir_prover(self, num_bytes: int) -> bytes:
        return shake256(self._prefix() + self.digest(), num_bytes)

    def fiat_shamir_verifier(self, num_bytes: int) -> bytes:
        return shake256(self._prefix() + serialize(self.objects[: self.read_index]), num_bytes)


# --------------------------------------------------------------------- FRI (L4)

class FRI:
    """fri.rs:13-416."""

    def __init__(self, offset: int, omega: int, domain_length: int, expansion_factor: int,
                 num_colinearity_tests: int):
        self.offset = offset
        self.omega = omega
        self.domain_length = domain_length
        self.expansion_factor = expansion_factor
        self.num_colinearity_tests = num_colinearity_tests

    def num_rounds(self) -> int:
        """fri.rs:40-50."""
        n = self.domain_length
        r = 0
        while n > self.expansion_factor and n > 4 * self.num_colinearity_tests:
            n //= 2
            r += 1
        return r

    def evaluate_domain(self) -> List[int]:
        """fri.rs:52-58."""
        return [mul_mod(self.offset, fpow(self.omega, i)) for i in range(self.domain_length)]

    @staticmethod
    def sample_index(data: bytes, size: int) -> int:
        """fri.rs:60-86: BE integer of the last floor(log2 size)/8 + 1 bytes, mod size."""
        assert size != 0, "modulo zero is impossible"
        nbytes = (size.bit_length() - 1) // 8 + 1
        tail = data[-nbytes:] if nbytes <= len(data) else data
        acc = 0
        for b in tail:
            acc = ((acc << 8) ^ b) & ((1 << 64) - 1)
        return acc % size

    def sample_indices(self, seed: bytes, size: int, reduced_size: int, number: int) -> List[int]:
        """fri.rs:88-113: blake2b(seed || 0^counter), reject duplicate reduced indices."""
        assert number <= 2 * reduced_size, "Not enough entropy in indices with reference to last codeword"
        assert number <= reduced_size, "Cannot sample more indices than available in the last codeword"
        indices, reduced = [], []
        counter = 0
        while len(indices) < number:
            index = self.sample_index(blake2b512(seed + bytes(counter)), size)
            r = index % reduced_size
            counter += 1
            if r not in reduced:
                indices.append(index)
                reduced.append(r)
        return indices

    @staticmethod
    def fold(codeword: Sequence[int], alpha: int, omega: int, offset: int) -> List[int]:
        """fri.rs:150-159: c'[i] = 2^-1 ((1 + a/(o w^i)) c[i] + (1 - a/(o w^i)) c[i + n/2])."""
        half = len(codeword) // 2
        two_inv = inv(2)
        out = []
        for i in range(half):
            abo = div(alpha, mul_mod(offset, fpow(omega, i)))
            first = mul_mod(add_mod(1, abo), codeword[i])
            second = mul_mod(sub_mod(1, abo), codeword[half + i])
            out.append(mul_mod(two_inv, add_mod(first, second)))
        return out

    def commit(self, codeword: Sequence[int], proof_stream: IndependentProofStream) -> List[List[int]]:
        """fri.rs:115-172: per round root -> push -> alpha = sample(FS) -> fold."""
        omega, offset = self.omega, self.offset
        rounds = self.num_rounds()
        codewords = []
        cw = list(codeword)
        for r in range(rounds):
            n = len(cw)
            assert fpow(omega, n - 1) == inv(omega), "error in commit: omega does not have the right order!"
            proof_stream.push((ROOT, merkle_commit(cw)))
            if r == rounds - 1:
                break
            alpha = sample(proof_stream.fiat_shamir_prover(PROOF_BYTES))
            codewords.append(list(cw))
            cw = self.fold(cw, alpha, omega, offset)
            omega = fpow(omega, 2)
            offset = fpow(offset, 2)
        proof_stream.push((CODEWORD, list(cw)))
        codewords.append(cw)
        return codewords

    def query(self, current: Sequence[int], nxt: Sequence[int], indices_c: Sequence[int],
              proof_stream: IndependentProofStream) -> List[int]:
        """fri.rs:174-208."""
        a = list(indices_c)
        b = [i + len(current) // 2 for i in indices_c]
        for s in range(self.num_colinearity_tests):
            proof_stream.push((LEAFS, (current[a[s]], current[b[s]], nxt[indices_c[s]])))
        lc, ln = merkle_levels(current), merkle_levels(nxt)
        for s in range(self.num_colinearity_tests):
            proof_stream.push((PATH, merkle_open_levels(a[s], lc)))
            proof_stream.push((PATH, merkle_open_levels(b[s], lc)))
            proof_stream.push((PATH, merkle_open_levels(indices_c[s], ln)))
        return a + b

    def prove(self, codeword: Sequence[int], proof_stream: IndependentProofStream) -> List[int]:
        """fri.rs:210-248."""
        assert self.domain_length == len(codeword), \
            "Length of the domain doesnt match the length of initial codeword"
        codewords = self.commit(codeword, proof_stream)
        top = self.sample_indices(proof_stream.fiat_shamir_prover(PROOF_BYTES), len(codewords[1]),
                                  len(codewords[-1]), self.num_colinearity_tests)
        indices = list(top)
        for i in range(len(codewords) - 1):
            el = codewords[i]
            indices = [j % (len(el) // 2) for j in indices]
            self.query(el, codewords[i + 1], indices, proof_stream)
        return top

    def verify(self, proof_stream: IndependentProofStream) -> Tuple[bool, str, List[Tuple[int, int]]]:
        """fri.rs:250-416 (returns (ok, error, polynomial_values))."""
        omega, offset = self.omega, self.offset
        rounds = self.num_rounds()
        roots, alphas = [], []
        points: List[Tuple[int, int]] = []
        for _ in range(rounds):
            code, root = proof_stream.pull()
            assert code == ROOT
            roots.append(root)
            alphas.append(sample(proof_stream.fiat_shamir_verifier(PROOF_BYTES)))
        code, last = proof_stream.pull()
        assert code == CODEWORD
        if merkle_commit(last) != roots[-1]:
            return False, "last codeword is not well formed", points
        degree = len(last) // self.expansion_factor - 1
        last_omega, last_offset = omega, offset
        for _ in range(rounds - 1):
            last_omega = fpow(last_omega, 2)
            last_offset = fpow(last_offset, 2)
        if inv(last_omega) != fpow(last_omega, len(last) - 1):
            return False, "omega does not have the right order", points
        poly = scale(intt(last_omega, last), inv(last_offset))
        nz = [i for i, c in enumerate(poly) if c != 0]
        if not nz:
            return False, "Received none instead of polynomial degree", points
        if nz[-1] > degree:
            return False, "last codeword does not correspond to polynomial of low enough degree", points
        if ntt(last_omega, scale(poly, last_offset)) != list(last):
            return False, "re-evaluated codeword does not match original", points
        top = self.sample_indices(proof_stream.fiat_shamir_verifier(PROOF_BYTES), self.domain_length >> 1,
                                  self.domain_length >> (rounds - 1), self.num_colinearity_tests)
        for r in range(rounds - 1):
            ic = [i % (self.domain_length >> (r + 1)) for i in top]
            ia = list(ic)
            ib = [i + (self.domain_length >> (r + 1)) for i in ia]
            aa, bb, cc = [], [], []
            for s in range(self.num_colinearity_tests):
                code, (ay, by, cy) = proof_stream.pull()
                assert code == LEAFS
                aa.append(ay)
                bb.append(by)
                cc.append(cy)
                if r == 0:
                    points.append((ia[s], ay))
                    points.append((ib[s], by))
                ax = mul_mod(offset, fpow(omega, ia[s]))
                bx = mul_mod(offset, fpow(omega, ib[s]))
                if not test_colinearity([(ax, ay), (bx, by), (alphas[r], cy)]):
                    return False, "colinearity check failure", points
            for i in range(self.num_colinearity_tests):
                for root, idx, leaf in ((roots[r], ia[i], aa[i]), (roots[r], ib[i], bb[i]),
                                        (roots[r + 1], ic[i], cc[i])):
                    code, path = proof_stream.pull()
                    assert code == PATH
                    if not merkle_verify(root, idx, path, leaf):
                        return False, "Merkle auth path verification failed", points
            omega = fpow(omega, 2)
            offset = fpow(offset, 2)
        return True, "", points


def test_colinearity(points: Sequence[Tuple[int, int]]) -> bool:
    """field/polynomial.rs:161-177: the interpolant through the points must have degree exactly 1.

    Equivalent closed form: all points on the line through the first two, and
    that line is not constant (a degree-0 interpolant is rejected).
    """
    (x0, y0), (x1, y1) = points[0], points[1]
    slope = div(sub_mod(y1, y0), sub_mod(x1, x0))
    for x, y in points[2:]:
        if add_mod(y0, mul_mod(slope, sub_mod(x, x0))) != y:
            return False
    return slope != 0


# ---------------------------------------------- synthetic workload generator

def synthetic_elements(seed: int, tag: bytes, n: int) -> List[int]:
    """SURVEY.md §8(d) value generator: 16-byte BE chunks of SHAKE256("sg-bench"||seed||tag) mod p."""
    stream = shake256(b"sg-bench" + seed.to_bytes(8, "big") + tag, 16 * n)
    return [int.from_bytes(stream[16 * i:16 * i + 16], "big") % P for i in range(n)]
