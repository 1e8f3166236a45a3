"""End-to-end SPARC simulation over AWGN (drop-in for sparc_public/sparc_sim.py).

sparc_sim(code_params, decode_params, awgn_var, rand_seed) returns the
reference's result dict (sparc_sim.py:8-58); the decoder runs on the GPU.
"""
import numpy as np

from .sparc import sparc_decode, sparc_encode


def sparc_sim(code_params, decode_params, awgn_var, rand_seed=None):
    """Encode, AWGN channel, AMP decode and error statistics (sparc_sim.py:8-58)."""
    bits_i, beta0, x, Ab, Az = sparc_encode(code_params, awgn_var, rand_seed)
    y = awgn_channel(x, awgn_var, rand_seed)
    bits_o, beta, T, nmse, expect = sparc_decode(y, code_params, decode_params, awgn_var, rand_seed,
                                                 beta0, Ab, Az)
    ber = calc_ber(bits_i, bits_o)
    cer = 1.0 * (ber > 0)
    detect = 1.0 * (not (ber > 0) ^ expect)
    results = {'ber': ber, 'cer': cer, 't_final': T, 'nmse': nmse, 'detect': detect}
    if code_params['modulated']:
        raise NotImplementedError("modulated SPARCs are not part of the GPU engine")
    ser, loc_of_sec_errs, num_of_sec_errs = calc_ser(beta0, beta, code_params['L'])
    results.update({'ser': ser, 'loc_of_sec_errs': loc_of_sec_errs,
                    'num_of_sec_errs': num_of_sec_errs})
    return results


def calc_ber(true_bin_array, est_bin_array):
    """Fraction of differing bits (sparc_sim.py:62-70)."""
    assert true_bin_array.dtype == 'bool'
    assert est_bin_array.dtype == 'bool'
    k = true_bin_array.size
    assert k == est_bin_array.size
    return np.count_nonzero(np.bitwise_xor(true_bin_array, est_bin_array)) / k


def calc_ser(beta0, beta, L):
    """Section error rate, error locations and count (sparc_sim.py:72-98)."""
    assert beta.size == beta0.size, 'beta and beta0 are of different size'
    assert beta.dtype == beta0.dtype, 'beta and beta0 are of different type'
    assert type(L) == int and L > 0
    assert beta.size % L == 0
    M = beta.size // L
    err = np.any(beta.reshape(L, M) != beta0.reshape(L, M), axis=1)
    num = int(np.count_nonzero(err))
    return num / L, np.flatnonzero(err), num


def awgn_channel(input_array, awgn_var, rand_seed):
    """y = x + N(0, awgn_var) from RandomState(rand_seed) (sparc_sim.py:179-204, real case)."""
    assert input_array.ndim == 1, 'input array must be one-dimensional'
    assert awgn_var >= 0
    rng = np.random.RandomState(rand_seed)
    n = input_array.size
    if input_array.dtype == np.float64:
        return input_array + np.sqrt(awgn_var) * rng.randn(n)
    if input_array.dtype == np.complex128:
        return input_array + np.sqrt(awgn_var / 2) * (rng.randn(n) + 1j * rng.randn(n))
    raise Exception("Unknown input type '{}'".format(input_array.dtype))
