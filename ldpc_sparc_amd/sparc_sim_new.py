"""End-to-end SPARC(+LDPC) simulation over AWGN (drop-in for
sparc_sophie/sparc_sim_new.py: sparc_ldpc_sim :12-23, the integrated-decoder
simulations :51-63, :65-75, :141-151, :154-164, awgn_channel :212-224).

The fork's *_test* simulations (diagnostic variants) are not provided
(SURVEY.md 2)."""
import numpy as np

from .sparc_new import (bit_err_rate, integrated_decoder, integrated_decoder_posteriors,
                        naively_integrated_decoder, naively_integrated_decoder_posteriors, sparc_ldpc_decode,
                        sparc_ldpc_encode)


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


def _sim(decoder, sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var, rand_seed):
    bits_i, total_bits, beta0, x, A = sparc_ldpc_encode(sparc_params, ldpc_params, lengths, ldpc_bool, rand_seed)
    y = awgn_channel(x, awgn_var, rand_seed)
    bits_o = decoder(y, sparc_params, ldpc_params, decode_params, A)
    return bits_i, bits_o, bit_err_rate(bits_i, bits_o)


def sparc_ldpc_naive_sim(sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var, rand_seed=None):
    """Encode, AWGN, naively_integrated_decoder (sparc_sim_new.py:51-63)."""
    return _sim(naively_integrated_decoder, sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var,
                rand_seed)


def sparc_ldpc_naive_sim_posteriors(sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var,
                                    rand_seed=None):
    """sparc_sim_new.py:65-75."""
    return _sim(naively_integrated_decoder_posteriors, sparc_params, ldpc_params, lengths, ldpc_bool, decode_params,
                awgn_var, rand_seed)


def sparc_ldpc_integrated_sim(sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var,
                              rand_seed=None):
    """Encode, AWGN, integrated_decoder (sparc_sim_new.py:141-151)."""
    return _sim(integrated_decoder, sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var,
                rand_seed)


def sparc_ldpc_integrated_posteriors_sim(sparc_params, ldpc_params, lengths, ldpc_bool, decode_params, awgn_var,
                                         rand_seed=None):
    """sparc_sim_new.py:154-164."""
    return _sim(integrated_decoder_posteriors, sparc_params, ldpc_params, lengths, ldpc_bool, decode_params,
                awgn_var, rand_seed)
