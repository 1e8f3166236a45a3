// Dense Gaussian-design AMP on gfx950 (sparc_sophie/sparc_new.py:885-912,
// msg_vector_mmse_estimator :1040-1066, MAP :1099-1116) and the AMP -> BP
// glue (beta_estimate_to_bp_probs :1118-1138, ldpc_bp :1167-1169).
//
// A batch of B codewords shares the design matrix A [n][LM], so the two
// matrix-vector products of the reference become GEMMs on the matrix cores:
//   A beta   : C[B][n]  = beta[B][LM] . A[n][LM]^T   (split over K = LM)
//   A^T z    : C[B][LM] = z[B][npad]  . A[n][LM]     (epilogue s = beta + C)
// f32 uses v_mfma_f32_32x32x2_f32 (exact f32 FMA chains); f64 (parity mode,
// small designs) uses plain FMA kernels.
#include "dense.hpp"
#include "philox.hpp"

namespace sg {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ f32 MFMA GEMM
// C[M][N] (+)= X[M][K] . Y, X K-contiguous; Y = [N][K] (NT) or [K][N] (NN).
// (64 MT) x 128 x 32 block tile, 4 waves in 2 x 2, each (32 MT) x 64 = MT x 2
// MFMA tiles.  MT = 4 covers a whole 256-codeword batch in one block row, so
// the design matrix (the Y operand, 19 GB at C5) is read once per launch; MT =
// 2 (128-row blocks) serves batches of at most 128.  Every output's k-order is
// the same for both (one MFMA chain over its K chunk), so they agree bit for bit.
struct GemmF32 {
    const float *X;
    long ldx;
    const float *Y;
    long ldy;
    float *C;
    long ldc;
    const float *add;  // NN epilogue: C = add + acc (same layout as C), or null
    long c_split;      // NT: split z writes C + z * c_split
    int M, N, K, kchunk, yrows;  // yrows: rows of Y (N for NT, K rows for NN) that exist
};

constexpr int GBN = 128, GBK = 32, GPAD = GBK + 1;

// The design-matrix operand (Y) is streamed once per launch; its loads can be
// non-temporal so that its lines leave the XCD's L2 first and the batch
// operand, which every N tile re-reads, stays resident (-DGEMM_Y_NT=0 for the A/B; on by default: 19.04 -> 18.91 ms per C5 GEMM launch same box, bit-identical).
#ifndef GEMM_Y_NT
#define GEMM_Y_NT 1
#endif
__device__ __forceinline__ float4 gemm_ld_y(const float *p) {
    if (GEMM_Y_NT) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const float4 *>(p);
}
template <int MT>
constexpr int gbm() { return 64 * MT; }
// Issue priority of a wave's MFMA loop (0: flat, for the A/B).  Two workgroups share a CU, so each SIMD
// runs one wave of each; at equal priority the older wave wins the issue arbitration, and a wave in its
// staging phase (LDS stores, barriers, next loads) held the MFMA pipe of the other one back.  The MFMA
// loop at 1 over a staging phase at 0: 18.88 -> 18.24 ms per C5 GEMM launch (0.833 -> 0.862 of the f32
// MFMA peak) same box, bit-identical; 2 and 3 measure the same (profiles/r05_prio_ab.txt).  Without the
// staging phase at all (barriers and LDS stores dropped, garbage results) the loop runs at 0.96.
#ifndef GEMM_PRIO
#define GEMM_PRIO 1
#endif

template <bool NT, int MT>
__global__ __launch_bounds__(256, MT == 4 ? 2 : 1) void gemm_f32_mfma(GemmF32 g) {  // (MT 4: 2 waves per SIMD)
    constexpr int BM = gbm<MT>(), XL = BM / 32;  // float4 loads of the X tile per thread
    __shared__ float Xs[BM * GPAD];
    __shared__ float Ys[NT ? GBN * GPAD : GBK * GBN];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * GBN;
    const int kb = blockIdx.z * g.kchunk;
    const int ke = min(g.K, kb + g.kchunk);
    const int nk = (ke - kb + GBK - 1) / GBK;
    float4 xr[XL], yr[4];
    auto load = [&](int k0) {
#pragma unroll
        for (int p = 0; p < XL; ++p) {
            const int f = tid + 256 * p;
            const int r = f >> 3, c = (f & 7) * 4;
            const int m = m0 + r;
            xr[p] = (m < g.M && k0 + c < ke) ? *reinterpret_cast<const float4 *>(g.X + (long)m * g.ldx + k0 + c)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int f = tid + 256 * p;
            if (NT) {
                const int r = f >> 3, c = (f & 7) * 4;
                const int nn = n0 + r;
                yr[p] = (nn < g.yrows && k0 + c < ke) ? gemm_ld_y(g.Y + (long)nn * g.ldy + k0 + c)
                                                      : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                const int r2 = f >> 5, c2 = (f & 31) * 4;
                const int kk = k0 + r2, nn = n0 + c2;
                yr[p] = (kk < ke && kk < g.yrows && nn < g.N) ? gemm_ld_y(g.Y + (long)kk * g.ldy + nn)
                                                               : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    f32x16 acc[MT][2];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    if (nk > 0) load(kb);
    for (int kt = 0; kt < nk; ++kt) {
        if (GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
#pragma unroll
        for (int p = 0; p < XL; ++p) {
            const int f = tid + 256 * p;
            const int r = f >> 3, c = (f & 7) * 4;
            float *xd = Xs + r * GPAD + c;
            xd[0] = xr[p].x; xd[1] = xr[p].y; xd[2] = xr[p].z; xd[3] = xr[p].w;
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int f = tid + 256 * p;
            if (NT) {
                const int r = f >> 3, c = (f & 7) * 4;
                float *yd = Ys + r * GPAD + c;
                yd[0] = yr[p].x; yd[1] = yr[p].y; yd[2] = yr[p].z; yd[3] = yr[p].w;
            } else {
                const int r2 = f >> 5, c2 = (f & 31) * 4;
                *reinterpret_cast<float4 *>(Ys + r2 * GBN + c2) = yr[p];
            }
        }
        __syncthreads();
        if (kt + 1 < nk) load(kb + (kt + 1) * GBK);  // next tile in flight during the MFMAs
        if (GEMM_PRIO) __builtin_amdgcn_s_setprio(GEMM_PRIO);
#pragma unroll
        for (int kk = 0; kk < GBK / 2; ++kk) {
            const int kx = 2 * kk + (lane >> 5);
            float a[MT], b[2];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) a[mt] = Xs[(wm * 32 * MT + mt * 32 + (lane & 31)) * GPAD + kx];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
                b[nt] = NT ? Ys[(wn * 64 + nt * 32 + (lane & 31)) * GPAD + kx]
                           : Ys[kx * GBN + wn * 64 + nt * 32 + (lane & 31)];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
        }
    }
    float *C = g.C + (long)blockIdx.z * g.c_split;
    // per 32 x 32 tile: the 16 addends requested together (clamped into the matrix, no branch), then the
    // 16 stores -- with the load inside each output's bounds branch, every output waited for its own
    // addend: 128 dependent round trips per thread at the end of each block
    const int rmax = g.M - 1, cmax = g.N - 1;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            float av[16];
            if (g.add) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * 32 * MT + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int col = n0 + wn * 64 + nt * 32 + (lane & 31);
                    av[r] = g.add[(long)min(row, rmax) * g.ldc + min(col, cmax)];
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 32 * MT + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int col = n0 + wn * 64 + nt * 32 + (lane & 31);
                if (row < g.M && col < g.N) {
                    const long o = (long)row * g.ldc + col;
                    C[o] = g.add ? av[r] + acc[mt][nt][r] : acc[mt][nt][r];
                }
            }
        }
}

// ------------------------------------------------------------------ f32 MFMA GEMM, LDS-DMA staging
// The same product and block tile with the operand tiles moved global -> LDS by global_load_lds_dwordx4
// (no staging registers, no LDS store instructions), K tiles of 16 in two LDS buffers: the DMA of tile t + 1
// is in flight while the MFMAs run on tile t, one barrier per tile.  A DMA writes 1 KiB per wave-instruction
// lane-linearly, so the conflict-free read layout comes from the source addresses: a 16-float row of the X
// (and NT Y) tile holds its four 16-byte groups at slot g ^ ((row >> 2) & 3), and each lane reads its 8
// k-values (k = 8 h + kk, h = lane >> 5, kk = 0..7: the MFMA's k pair at step kk is {kk, 8 + kk}) as two
// ds_read_b128 -- 16 consecutive rows of one read cover all 16 slots of a bank row.  The NN Y tile ([k][n],
// 512-byte rows) is read along n as before.  Every output's k order is the same for both MT, so the two
// block heights still agree bit for bit (a different order from gemm_f32_mfma's, so not with it).
// Needs tiles without ragged K (the K chunk a multiple of 16) and, for NN, N a multiple of 128; rows past M
// or past yrows read a clamped row (their products land in unstored outputs, or meet z's zero padding).
constexpr int GBK2 = 16;
// the LDS-DMA kernel where its tiles are whole (1), or the register-staged kernel everywhere (0) (A/B): C5 GEMM
// 0.864 -> 0.868 / 0.871 of the f32 MFMA peak same box, the C5 and dense tests green
// (profiles/r06_gemm_glds_ab.txt)
#ifndef GEMM_GLDS
#define GEMM_GLDS 1
#endif
template <int MT>
constexpr int glds_buf_floats() { return 64 * MT * GBK2 + GBN * GBK2; }  // one buffer: the X and Y tiles
typedef __attribute__((address_space(3))) void lds_void;
// one 16-byte-per-lane DMA global -> LDS (buffer_load_dwordx4 ... lds): lane i's 16 bytes land at lds + 16 i
// (a non-template device function: the builtin inside the kernel template kept the host pass from emitting its
// launch stubs)
template <int AUX>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, float *lds, int vo, int so) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)lds, 16, vo, so, 0, AUX);
}
// the design matrix's DMAs non-temporal (aux 2: nt), as gemm_ld_y's loads, so the streamed A leaves the XCD's L2
// before the batch operand every N tile re-reads (1), or default policy (0) (A/B).  Same box: default 0.873 / 0.872
// of the f32 MFMA peak, nt 0.866 / 0.865 (the register-staged kernel 0.866 / 0.865); fabric bytes per NT launch
// 37.5 GB (default) / 41.0 GB (nt): the batch operand is re-read past L2 either way, and the GEMM is MFMA-bound
// (A once is 19.3 GB, 2.4 ms of an 18 ms launch at 8 TB/s) (profiles/r06_gemm_glds_ab.txt)
#ifndef GEMM_GLDS_YNT
#define GEMM_GLDS_YNT 0
#endif
constexpr int GLDS_YAUX = GEMM_GLDS_YNT ? 2 : 0;
template <bool NT, int MT>
__global__ __launch_bounds__(256, MT == 4 ? 2 : 1) void gemm_f32_glds(GemmF32 g) {
    constexpr int BM = gbm<MT>(), BUF = glds_buf_floats<MT>();
    __shared__ __attribute__((aligned(16))) float lds[2 * BUF];  // two buffers, one LDS object
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * GBN;
    const int kb = blockIdx.z * g.kchunk;
    const int ke = min(g.K, kb + g.kchunk);
    const int nk = (ke - kb) / GBK2;
    // DMA sources through buffer resources based at the block's first row (32-bit per-lane offsets; rows
    // past M / yrows are past the resource's end and read as 0)
    // (every resource field through readfirstlane: a resource the compiler cannot prove uniform gets a waterfall
    // loop around each DMA)
    const int ldx = __builtin_amdgcn_readfirstlane((int)g.ldx), ldy = __builtin_amdgcn_readfirstlane((int)g.ldy);
    const int nrx = __builtin_amdgcn_readfirstlane(4 * ldx * max(0, min(BM, g.M - m0)));
    const int nry = __builtin_amdgcn_readfirstlane(4 * ldy * max(0, min(GBN, g.yrows - n0)));
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(g.X + (long)m0 * ldx), 0, nrx, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(g.Y + (long)n0 * ldy), 0, nry, 0x00020000);
    // per-lane source offsets (tile-invariant) and the wave's LDS destinations
    int ox[BM / 64], oy[2];
#pragma unroll
    for (int i = 0; i < BM / 64; ++i) {
        const int row = 16 * (i * 4 + wid) + (lane >> 2);
        ox[i] = 4 * row * ldx + 16 * ((lane & 3) ^ ((row >> 2) & 3));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (NT) {
            const int row = 16 * (i * 4 + wid) + (lane >> 2);
            oy[i] = 4 * row * ldy + 16 * ((lane & 3) ^ ((row >> 2) & 3));
        } else {
            oy[i] = 4 * (2 * (i * 4 + wid) + (lane >> 5)) * ldy + 16 * (lane & 31);
        }
    }
    auto stage = [&](int buf, int k0) {
        float *bx = lds + buf * BUF, *by = bx + BM * GBK2;
        // X: BM rows x 4 slots = BM / 16 wave-instructions of 16 rows
#pragma unroll
        for (int i = 0; i < BM / 64; ++i)
            dma16<0>(rx, bx + 256 * (i * 4 + wid), ox[i], 4 * k0);
        if (NT) {  // 128 n-rows x 4 slots
#pragma unroll
            for (int i = 0; i < 2; ++i)
                dma16<GLDS_YAUX>(ry, by + 256 * (i * 4 + wid), oy[i], 4 * k0);
        } else {  // 16 k-rows x 128 n, two k-rows per wave-instruction (A is 19 GB at C5: a resource per tile)
            const int nrk = __builtin_amdgcn_readfirstlane(4 * ldy * max(0, min(GBK2, g.yrows - k0)));
            const __amdgpu_buffer_rsrc_t rk =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(g.Y + (long)k0 * ldy + n0), 0, nrk, 0x00020000);
#pragma unroll
            for (int i = 0; i < 2; ++i)
                dma16<GLDS_YAUX>(rk, by + 256 * (i * 4 + wid), oy[i], 0);
        }
    };
    f32x16 acc[MT][2];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    const int h = lane >> 5, rl = lane & 31;
    // a tile's fragments in registers (k = 8 h + 4 q + 0..3)
    struct Frag {
        float4 a[MT][2], b[2][2];
        float bn[2][GBK2 / 2];
    };
    auto read_frag = [&](const float *bx, Frag &f) {
        const float *by = bx + BM * GBK2;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int row = wm * 32 * MT + mt * 32 + rl;
                f.a[mt][q] = *reinterpret_cast<const float4 *>(bx + 16 * row + 4 * ((2 * h + q) ^ ((row >> 2) & 3)));
            }
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                if (NT) {
                    const int row = wn * 64 + nt * 32 + rl;
                    f.b[nt][q] = *reinterpret_cast<const float4 *>(by + 16 * row + 4 * ((2 * h + q) ^ ((row >> 2) & 3)));
                } else {
#pragma unroll
                    for (int k4 = 0; k4 < 4; ++k4)
                        f.bn[nt][4 * q + k4] = by[(8 * h + 4 * q + k4) * GBN + wn * 64 + nt * 32 + rl];
                }
            }
        }
    };
    auto mma = [&](const Frag &f, int q) {  // the MFMAs of k4 = 0..3 of half q of the tile
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            float a[MT], b[2];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const float4 v = f.a[mt][q];
                a[mt] = k4 == 0 ? v.x : k4 == 1 ? v.y : k4 == 2 ? v.z : v.w;
            }
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                if (NT) {
                    const float4 v = f.b[nt][q];
                    b[nt] = k4 == 0 ? v.x : k4 == 1 ? v.y : k4 == 2 ? v.z : v.w;
                } else {
                    b[nt] = f.bn[nt][4 * q + k4];
                }
            }
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
        }
    };
    if (nk > 0) stage(0, kb);
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt landed (the barrier's fence waits for this wave's DMAs), and every wave has read its fragments
        // of tile kt - 1, so the other buffer is free
        if (GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        // the whole tile's fragments first, THEN the next tile's DMA: with a DMA in flight the compiler waits
        // vmcnt(0) before any LDS read of the same object
        Frag f;
        read_frag(lds + (kt & 1) * BUF, f);
        if (kt + 1 < nk) stage((kt + 1) & 1, kb + (kt + 1) * GBK2);
        if (GEMM_PRIO) __builtin_amdgcn_s_setprio(GEMM_PRIO);
        mma(f, 0);
        mma(f, 1);
    }
    float *C = g.C + (long)blockIdx.z * g.c_split;
    const int rmax = g.M - 1, cmax = g.N - 1;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            float av2[16];
            if (g.add) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * 32 * MT + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int col = n0 + wn * 64 + nt * 32 + (lane & 31);
                    av2[r] = g.add[(long)min(row, rmax) * g.ldc + min(col, cmax)];
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 32 * MT + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int col = n0 + wn * 64 + nt * 32 + (lane & 31);
                if (row < g.M && col < g.N) {
                    const long o = (long)row * g.ldc + col;
                    C[o] = g.add ? av2[r] + acc[mt][nt][r] : acc[mt][nt][r];
                }
            }
        }
}

// the LDS-DMA kernel (1) or the register-staged one (0) (A/B); the DMA kernel only where its tiles are whole
static bool glds_ok(const GemmF32 &g, bool nt) {
    // whole K tiles, 16-byte aligned rows (aligned bases, row strides of 4 floats), whole NN column tiles,
    // 32-bit per-block offsets
    return GEMM_GLDS && g.K % GBK2 == 0 && g.kchunk % GBK2 == 0 && g.ldx % 4 == 0 && g.ldy % 4 == 0 &&
           ((uintptr_t)g.X % 16 == 0) && ((uintptr_t)g.Y % 16 == 0) &&
           (nt || g.N % GBN == 0) && g.M > 0 && g.yrows > 0 && 4.0 * g.ldx * gbm<4>() < 2147483647.0 &&
           4.0 * g.ldy * GBN < 2147483647.0;
}

// Block rows of 256 once the batch exceeds 128 codewords (A read ceil(B / 256)
// times instead of ceil(B / 128)); 128 below that (no idle half tile).
template <bool NT>
static void gemm_launch(const GemmF32 &g, unsigned gx, unsigned gz, hipStream_t s) {
    if (glds_ok(g, NT)) {
        if (g.M > gbm<2>())
            hipLaunchKernelGGL((gemm_f32_glds<NT, 4>), dim3(gx, (g.M + gbm<4>() - 1) / gbm<4>(), gz), dim3(256), 0, s, g);
        else
            hipLaunchKernelGGL((gemm_f32_glds<NT, 2>), dim3(gx, (g.M + gbm<2>() - 1) / gbm<2>(), gz), dim3(256), 0, s, g);
        return;
    }
    if (g.M > gbm<2>())
        hipLaunchKernelGGL((gemm_f32_mfma<NT, 4>), dim3(gx, (g.M + gbm<4>() - 1) / gbm<4>(), gz), dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL((gemm_f32_mfma<NT, 2>), dim3(gx, (g.M + gbm<2>() - 1) / gbm<2>(), gz), dim3(256), 0, s, g);
}

// ------------------------------------------------------------------ f64 (parity) products
// part[0][b][i] = sum_j A[i][j] beta[b][j]: one workgroup per row i.
__global__ __launch_bounds__(256) void ab_f64_kernel(const double *__restrict__ A, const double *__restrict__ beta,
                                                     int n, int LM, int B, double *__restrict__ out) {
    __shared__ double red[4][8];
    const int i = blockIdx.x, tid = threadIdx.x;
    const double *Ai = A + (long)i * LM;
    for (int b0 = 0; b0 < B; b0 += 8) {
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int j = tid; j < LM; j += 256) {
            const double a = Ai[j];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (b0 + q < B) acc[q] += a * beta[(long)(b0 + q) * LM + j];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            double v = acc[q];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if ((tid & 63) == 0) red[tid >> 6][q] = v;
        }
        __syncthreads();
        if (tid < 8 && b0 + tid < B)
            out[(long)(b0 + tid) * n + i] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
        __syncthreads();
    }
}

// s[b][j] = beta[b][j] + sum_i A[i][j] z[b][i]
__global__ __launch_bounds__(256) void az_f64_kernel(const double *__restrict__ A, const double *__restrict__ z,
                                                     const double *__restrict__ beta, int n, int npad, int LM,
                                                     double *__restrict__ s) {
    const int b = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= LM) return;
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += A[(long)i * LM + j] * z[(long)b * npad + i];
    s[(long)b * LM + j] = beta[(long)b * LM + j] + acc;
}

// ------------------------------------------------------------------ residual
// t > 0: z = y - A beta + (z / tau^2)(P - ||beta||^2 / n)   (sparc_new.py:902-905)
// t = 0: z = y.  Also writes per-block partial sums of z^2 for tau^2.
template <typename T>
__global__ __launch_bounds__(256) void residual_kernel(DenseBufs<T> d, int t, double *z2part, int nblk) {
    __shared__ double red[4];
    __shared__ double sh_bsq;
    const int b = blockIdx.y, tid = threadIdx.x;
    const int i = blockIdx.x * 256 + tid;
    if (t > 0 && d.ons_mode == 0 && tid < 64) {  // ||beta||^2 of the codeword, fixed order
        double v = 0.0;
        for (int l = tid; l < d.L; l += 64) v += d.sec_bsq[(long)b * d.L + l];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (tid == 0) sh_bsq = v;
    }
    __syncthreads();
    double zz = 0.0;
    if (i < d.npad) {
        T zn = T(0);
        if (i < d.n) {
            const T y = d.y[(long)b * d.n + i];
            if (t > 0) {
                T r = T(0);
                for (int sp = 0; sp < d.nsplit; ++sp) r += d.part[((long)sp * d.B + b) * d.n + i];
                const T zo = d.z[(long)b * d.npad + i];
                T ons;
                if (d.ons_mode == 1) ons = (zo / (T)d.n) * (T)d.ons[b];
                else if (d.ons_mode == 2) ons = zo * (T)(d.ons[b] / d.n);
                else ons = (zo / (T)d.tau2[b]) * (T)(d.P - sh_bsq / d.n);
                zn = (y - r) + ons;
            } else {
                zn = y;
            }
        }
        d.z[(long)b * d.npad + i] = zn;
        zz = (double)zn * (double)zn;
    }
    for (int o = 32; o > 0; o >>= 1) zz += __shfl_xor(zz, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = zz;
    __syncthreads();
    if (tid == 0) z2part[(long)b * nblk + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void tau2_kernel(const double *z2part, int nblk, int n, double *tau2) {
    const int b = blockIdx.x;
    if (threadIdx.x == 0) {
        double v = 0.0;
        for (int k = 0; k < nblk; ++k) v += z2part[(long)b * nblk + k];
        tau2[b] = v / n;  // tau_sqr = sum(z^2) / n (sparc_new.py:908)
    }
}

// ------------------------------------------------------------------ eta
// beta = sqrt(n P_l) softmax(sqrt(n P_l) s / tau^2) per section (sparc_new.py:1058-1066,
// per-section maximum: same value as the reference's global shift), and the
// section's sum of beta^2.  One wavefront per section.
template <typename T>
__device__ __forceinline__ T dexp2(T x);
template <>
__device__ __forceinline__ float dexp2<float>(float x) { return __expf(x); }
template <>
__device__ __forceinline__ double dexp2<double>(double x) { return exp(x); }

constexpr int DETA_R = 16;  // entries per lane held in registers (sections of M <= 1024)
template <typename T>
__global__ __launch_bounds__(256) void dense_eta_kernel(DenseBufs<T> d) {
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = blockIdx.y;
    if (l >= d.L) return;
    const double snp = sqrt((double)d.n * (d.P / d.L));
    const T c = (T)snp, tau2 = (T)d.tau2[b];
    const T *s = d.s + (long)b * d.LM + (long)l * d.M;
    T *beta = d.beta + (long)b * d.LM + (long)l * d.M;
    T mx = -INFINITY;
    double sq = 0.0;
    if (d.M <= 64 * DETA_R) {
        // the section in registers: s read once, its exponent argument and exponential computed
        // once per entry (the loop form below re-reads s and recomputes both in every pass);
        // the same per-entry values and per-lane summation order
        T x[DETA_R];
#pragma unroll
        for (int r = 0; r < DETA_R; ++r) {
            const int j = lane + 64 * r;
            x[r] = j < d.M ? c * (s[j] / tau2) : T(-INFINITY);
        }
#pragma unroll
        for (int r = 0; r < DETA_R; ++r) mx = fmax(mx, x[r]);
        for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
        T den = T(0);
#pragma unroll
        for (int r = 0; r < DETA_R; ++r) {
            x[r] = lane + 64 * r < d.M ? dexp2<T>(x[r] - mx) : T(0);
            den += x[r];
        }
        for (int o = 32; o > 0; o >>= 1) den += __shfl_xor(den, o, 64);
#pragma unroll
        for (int r = 0; r < DETA_R; ++r) {
            const int j = lane + 64 * r;
            if (j < d.M) {
                const T v = c * (x[r] / den);
                beta[j] = v;
                sq += (double)v * (double)v;
            }
        }
    } else {
        for (int j = lane; j < d.M; j += 64) mx = fmax(mx, c * (s[j] / tau2));
        for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
        T den = T(0);
        for (int j = lane; j < d.M; j += 64) den += dexp2<T>(c * (s[j] / tau2) - mx);
        for (int o = 32; o > 0; o >>= 1) den += __shfl_xor(den, o, 64);
        for (int j = lane; j < d.M; j += 64) {
            const T v = c * (dexp2<T>(c * (s[j] / tau2) - mx) / den);
            beta[j] = v;
            sq += (double)v * (double)v;
        }
    }
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (lane == 0) d.sec_bsq[(long)b * d.L + l] = sq;
}

// Per-section sum of beta^2 of a given beta (state handed in by the caller).
template <typename T>
__global__ __launch_bounds__(256) void dense_bsq_kernel(DenseBufs<T> d) {
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = blockIdx.y;
    if (l >= d.L) return;
    const T *beta = d.beta + (long)b * d.LM + (long)l * d.M;
    double sq = 0.0;
    for (int j = lane; j < d.M; j += 64) sq += (double)beta[j] * (double)beta[j];
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (lane == 0) d.sec_bsq[(long)b * d.L + l] = sq;
}

template <typename T>
int dense_launch_bsq(const DenseBufs<T> &d, hipStream_t s) {
    hipLaunchKernelGGL((dense_bsq_kernel<T>), dim3((d.L + 3) / 4, d.B), dim3(256), 0, s, d);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

// MAP: first index of the section maximum of s (numpy argmax).
template <typename T>
__global__ __launch_bounds__(256) void dense_map_kernel(const T *s, int B, int L, int M, int32_t *idx) {
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = blockIdx.y;
    if (l >= L) return;
    const T *ss = s + (long)b * L * M + (long)l * M;
    T best = -INFINITY;
    int arg = 0x7fffffff;
    for (int j = lane; j < M; j += 64)
        if (arg == 0x7fffffff || ss[j] > best) { best = ss[j]; arg = j; }
    T g = best;
    for (int o = 32; o > 0; o >>= 1) g = fmax(g, __shfl_xor(g, o, 64));
    int cand = (best == g) ? arg : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    if (lane == 0) idx[(long)b * L + l] = cand == 0x7fffffff ? 0 : cand;
}

// ------------------------------------------------------------------ glue
// LLR of each (MSB-first) bit of the protected sections from the soft
// estimate: p0 = sum over indices whose bit is 0 of beta / sqrt(n P_l),
// clipped to [1e-15, 1 - 1e-15], LLR = log p0 - log(1 - p0) (positive => 0).
template <typename T>
__global__ __launch_bounds__(256) void glue_llr_kernel(const T *beta, int B, int L, int M, int l0, int nl,
                                                       double inv_snp, int llr_ld, T *llr, int probs_only) {
    const int lane = threadIdx.x & 63;
    const int li = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = blockIdx.y;
    if (li >= nl) return;
    int logM = 0;
    while ((1 << logM) < M) ++logM;
    const T *bs = beta + (long)b * L * M + (long)(l0 + li) * M;
    for (int pos = 0; pos < logM; ++pos) {
        const int bit = logM - 1 - pos;
        double p = 0.0;
        for (int j = lane; j < M; j += 64)
            if (((j >> bit) & 1) == 0) p += (double)bs[j] * inv_snp;
        for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
        if (lane == 0) {
            const double eps = 1e-15;
            const double pc = fmin(fmax(p, eps), 1.0 - eps);  // ldpc_bp's clip (sparc_new.py:1167)
            llr[(long)b * llr_ld + (long)li * logM + pos] = probs_only ? (T)p : (T)(log(pc) - log(1.0 - pc));
        }
    }
}

// ------------------------------------------------------------------ concatenated error counts
// Per codeword (sparc_sim_new.py:21, bit_err_rate): unprotected bits from the
// MAP section indices (MSB-first bits of the index, sparc_new.py:1319-1341),
// protected bits = hard decisions app[:K] < 0 of every LDPC block
// (sparc_new.py:1185-1187).  Adds {codewords, bit errors, codeword errors,
// unprotected bit errors, protected bit errors} to counts[5].
template <typename T>
__global__ __launch_bounds__(256) void concat_count_kernel(const int32_t *map_idx, const int32_t *true_idx, int L,
                                                           int L_unp, int logM, const T *app, const uint8_t *info,
                                                           int mults, int N, int K, unsigned long long *counts) {
    __shared__ int red[2][4];
    const int cw = blockIdx.x, tid = threadIdx.x;
    int eu = 0, ep = 0;
    const unsigned mask = (1u << logM) - 1u;
    for (int l = tid; l < L_unp; l += blockDim.x)
        eu += __popc(((unsigned)map_idx[(long)cw * L + l] ^ (unsigned)true_idx[(long)cw * L + l]) & mask);
    for (int e = tid; e < mults * K; e += blockDim.x) {
        const int blk = e / K, v = e - blk * K;
        const int hard = app[((long)cw * mults + blk) * N + v] < T(0) ? 1 : 0;
        ep += hard != (int)info[(long)cw * mults * K + e];
    }
    for (int o = 32; o > 0; o >>= 1) {
        eu += __shfl_xor(eu, o, 64);
        ep += __shfl_xor(ep, o, 64);
    }
    if ((tid & 63) == 0) { red[0][tid >> 6] = eu; red[1][tid >> 6] = ep; }
    __syncthreads();
    if (tid == 0) {
        int u = 0, q = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { u += red[0][w]; q += red[1][w]; }
        atomicAdd(&counts[0], 1ull);
        atomicAdd(&counts[1], (unsigned long long)(u + q));
        atomicAdd(&counts[2], (unsigned long long)(u + q > 0));
        atomicAdd(&counts[3], (unsigned long long)u);
        atomicAdd(&counts[4], (unsigned long long)q);
    }
}

template <typename T>
int concat_launch_count(const int32_t *map_idx, const int32_t *true_idx, int B, int L, int L_unp, int logM,
                        const T *app, const uint8_t *info, int mults, int N, int K, int64_t *counts, hipStream_t s) {
    if (B <= 0) return SG_OK;
    hipLaunchKernelGGL((concat_count_kernel<T>), dim3(B), dim3(256), 0, s, map_idx, true_idx, L, L_unp, logM, app,
                       info, mults, N, K, reinterpret_cast<unsigned long long *>(counts));
    SG_HIP(hipGetLastError());
    return SG_OK;
}

// ------------------------------------------------------------------ random design
// Throughput mode: A[i][j] ~ N(0, 1/n) from Philox4x32-10 (counter = element
// index / 4, key = seed) and Box-Muller; statistically, not bitwise, equal to
// numpy's default_rng(seed).normal (parity mode uploads the reference draw).
template <typename T>
__global__ void gen_A_kernel(T *A, long total, double scale, uint64_t seed) {
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;  // 4 outputs per thread
    if (q * 4 >= total) return;
    uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), 0x5eed5eedu, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double two32 = 4294967296.0;
    float out[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const double u1 = ((double)c[2 * h] + 1.0) / (two32 + 1.0);
        const double u2 = (double)c[2 * h + 1] / two32;
        const double r = sqrt(-2.0 * log(u1));
        out[2 * h] = (float)(r * cos(2.0 * M_PI * u2));
        out[2 * h + 1] = (float)(r * sin(2.0 * M_PI * u2));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (q * 4 + e < total) A[q * 4 + e] = (T)(out[e] * scale);
}

// ------------------------------------------------------------------ launchers
template <>
int dense_launch_ab<float>(const DenseBufs<float> &d, hipStream_t s) {
    ProfScope ps(SG_PH_DENSE, s);
    GemmF32 g;
    g.X = d.beta; g.ldx = d.LM; g.Y = d.A; g.ldy = d.LM; g.C = d.part; g.ldc = d.n; g.add = nullptr;
    g.c_split = (long)d.B * d.n; g.M = d.B; g.N = d.n; g.K = d.LM; g.yrows = d.n;
    g.kchunk = ((d.LM + d.nsplit - 1) / d.nsplit + GBK - 1) / GBK * GBK;
    gemm_launch<true>(g, (d.n + GBN - 1) / GBN, d.nsplit, s);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <>
int dense_launch_ab<double>(const DenseBufs<double> &d, hipStream_t s) {
    ProfScope ps(SG_PH_DENSE, s);
    hipLaunchKernelGGL(ab_f64_kernel, dim3(d.n), dim3(256), 0, s, d.A, d.beta, d.n, d.LM, d.B, d.part);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <>
int dense_launch_az<float>(const DenseBufs<float> &d, hipStream_t s) {
    ProfScope ps(SG_PH_DENSE, s);
    GemmF32 g;
    g.X = d.z; g.ldx = d.npad; g.Y = d.A; g.ldy = d.LM; g.C = d.s; g.ldc = d.LM; g.add = d.beta;
    g.c_split = 0; g.M = d.B; g.N = d.LM; g.K = d.npad; g.kchunk = d.npad; g.yrows = d.n;
    gemm_launch<false>(g, (d.LM + GBN - 1) / GBN, 1, s);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <>
int dense_launch_az<double>(const DenseBufs<double> &d, hipStream_t s) {
    ProfScope ps(SG_PH_DENSE, s);
    hipLaunchKernelGGL(az_f64_kernel, dim3((d.LM + 255) / 256, d.B), dim3(256), 0, s, d.A, d.z, d.beta, d.n, d.npad,
                       d.LM, d.s);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int dense_launch_residual(const DenseBufs<T> &d, int t, hipStream_t s) {
    ProfScope ps(SG_PH_CONTROL, s);
    const int nblk = (d.npad + 255) / 256;
    double *z2part = d.tau2 + d.B;  // the plan allocates tau2 with B + B * nblk entries
    hipLaunchKernelGGL((residual_kernel<T>), dim3(nblk, d.B), dim3(256), 0, s, d, t, z2part, nblk);
    hipLaunchKernelGGL(tau2_kernel, dim3(d.B), dim3(64), 0, s, z2part, nblk, d.n, d.tau2);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int dense_launch_eta(const DenseBufs<T> &d, hipStream_t s) {
    ProfScope ps(SG_PH_ETA, s);
    hipLaunchKernelGGL((dense_eta_kernel<T>), dim3((d.L + 3) / 4, d.B), dim3(256), 0, s, d);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int dense_launch_gen_A(T *A, int n, int LM, uint64_t seed, hipStream_t s) {
    const long total = (long)n * LM;
    const long nthr = (total + 3) / 4;
    hipLaunchKernelGGL((gen_A_kernel<T>), dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s, A, total,
                       1.0 / sqrt((double)n), seed);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int dense_launch_map(const T *sv, int B, int L, int M, int32_t *idx, hipStream_t s) {
    hipLaunchKernelGGL((dense_map_kernel<T>), dim3((L + 3) / 4, B), dim3(256), 0, s, sv, B, L, M, idx);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int glue_launch_llr(const T *beta, int B, int L, int M, int l0, int nl, double inv_snp, int llr_ld, T *llr,
                    int probs_only, hipStream_t s) {
    if (B <= 0 || nl <= 0) return SG_OK;
    hipLaunchKernelGGL((glue_llr_kernel<T>), dim3((nl + 3) / 4, B), dim3(256), 0, s, beta, B, L, M, l0, nl, inv_snp,
                       llr_ld, llr, probs_only);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

#define SG_DENSE_INST(T)                                                                                        \
    template int dense_launch_bsq<T>(const DenseBufs<T> &, hipStream_t);                                       \
    template int concat_launch_count<T>(const int32_t *, const int32_t *, int, int, int, int, const T *,        \
                                        const uint8_t *, int, int, int, int64_t *, hipStream_t);              \
    template int dense_launch_residual<T>(const DenseBufs<T> &, int, hipStream_t);                             \
    template int dense_launch_eta<T>(const DenseBufs<T> &, hipStream_t);                                       \
    template int dense_launch_gen_A<T>(T *, int, int, uint64_t, hipStream_t);                                  \
    template int dense_launch_map<T>(const T *, int, int, int, int32_t *, hipStream_t);                        \
    template int glue_launch_llr<T>(const T *, int, int, int, int, int, double, int, T *, int, hipStream_t);
SG_DENSE_INST(float)
SG_DENSE_INST(double)

}  // namespace sg
