"""End-to-end SPARC(+LDPC) simulation over AWGN (drop-in for
sparc_sophie/sparc_sim_new.py: sparc_ldpc_sim :12-23, awgn_channel :212-224).

The fork's other *_sim* variants wrap its experimental decoders and are not
provided."""
import numpy as np

from .sparc_new import bit_err_rate, sparc_ldpc_decode, sparc_ldpc_encode


def sparc_ldpc_sim(sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var, rand_seed=None):
    """Encode, AWGN, decode (AMP then BP), BER.  Returns (bits_in, bits_out, ber)."""
    bits_i, total_bits, beta0, x, A = sparc_ldpc_encode(sparc_params, ldpc_params, lengths, ldpc_bool, rand_seed)
    y = awgn_channel(x, awgn_var, rand_seed)
    bits_o = sparc_ldpc_decode(y, sparc_params, ldpc_params, decode_params, ldpc_bool, lengths, A)
    ber = bit_err_rate(bits_i, bits_o)
    return bits_i, bits_o, ber


def awgn_channel(input_array, awgn_var, rand_seed):
    """y = x + sqrt(awgn_var) RandomState(rand_seed).randn(n)."""
    assert input_array.ndim == 1, 'input array must be one-dimensional'
    assert awgn_var >= 0
    rng = np.random.RandomState(rand_seed)
    n = input_array.size
    return input_array + np.sqrt(awgn_var) * rng.randn(n)
