"""C5 probe for the profilers: the bench's concatenated pipeline (n = 9216,
B = 256, Eb/N0 5.5 dB, batch generated on the GPU) decoded `reps` times."""
import sys

sys.path.insert(0, ".")
from ldpc_sparc_amd import _native  # noqa: E402
from ldpc_sparc_amd.pipeline import ConcatPipeline  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
L, M, n, P, Lu, mults, B = 1024, 512, 9216, 15.0, 160, 4, 256
pipe = ConcatPipeline(L, M, n, P, Lu, mults, design_seed=1234, precision="f32", t_max=25)
R = (Lu * 9 + mults * pipe.c.K) / n
var = P / (2 * R * 10 ** (5.5 / 10))
pipe.make_batch_device(B, var, 5000, 0)
for _ in range(reps):
    pipe.reset_counts()
    pipe.decode()
_native.device_synchronize()
print("counts", pipe.counts().tolist())
