"""starkgpu: MI355X-native LDE / NTT / Merkle / FRI-commit hot path of the
"Anatomy of a STARK" prover (SpekalsG3/zk-stark-tutor), behind the C ABI in
include/stark_gpu.h.  See DESIGN.md."""
from ._lib import LIB_PATH, StarkGpuError, lib
from .api import (CODEWORD, FIELD_PRIME, LEAFS, PATH, PROOF_BYTES, ROOT, VALUE, CallbackProofStream, Context, HostContext,
                  DeviceTree, FRI, IndependentProofStream, MerkleRoot, SignatureProofStream, decode_object,
                  encode_object, fast_coset_evaluate, fast_coset_evaluate_batch_dev,
                  fast_coset_evaluate_dev, fe_array, fe_inverse, fe_mul, fe_pow,
                  generator, intt, intt_dev, ntt, ntt_dev, primitive_nth_root, sample, to_ints)

from .algebra import (Polynomial, fast_coset_divide, fast_interpolate_domain, fast_interpolate_geometric_dev,
                      fast_multiply, fast_zerofier, fast_zerofier_geometric)
from .stark import MPolynomial, RescuePrime, Stark

__all__ = [n for n in dir() if not n.startswith("_")]
