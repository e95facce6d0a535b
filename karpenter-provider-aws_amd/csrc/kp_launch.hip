// kp_launch.hip — launch-time instance-type selection on gfx950: one 256-thread workgroup per NodeClaim launch request.
//
// Restates, per request (pkg/providers/instance/instance.go:132-137, 270-298, 420-467, 532-546):
//   the filter chain of pkg/providers/instance/filter/filter.go in its fixed order
//     CompatibleAvailable :39-64 → CapacityReservationType :73-157 → CapacityBlock :163-221 →
//     ReservedOffering :230-270 → ExoticInstanceType :279-318 → SpotInstance :328-386,
//   a filter that leaves nothing = ICE (instance.go:281-284); [core] InstanceTypes.Truncate(reqs, M) = OrderByPrice
//   (cheapest Available().Compatible(reqs) offering, MaxFloat64 when none, ties by name) + first M + SatisfiesMinValues;
//   getCapacityType (reserved > spot > on-demand, requirements narrowed to that capacity type);
//   getOverrides' offering side (Available ∧ Compatible with capacity-type := chosen).
//
// Layout: the workgroup's threads own types t ≡ tid (mod 256).  Per type the LDS holds u64 masks over its offerings
// (≤ 64): lv = the offerings the filters left on it (it.Offerings), cmn = Compatible on every offering key but
// capacity-type, ctok = Compatible on capacity-type, am = Available.  Offering filters rewrite lv in place, exactly as
// the reference rewrites it.Offerings.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cfloat>

#include "../../include/kpsim.h"
#include "kp_launch.h"
#include "kp_layout.h"
#include "kp_wave.h"

namespace {

constexpr int NT = 256;
constexpr int NWV = NT / 64;

struct LShared {  // reductions (static LDS)
    double redd[NWV];
    int redi[NWV];
    int ncomp;
};

// Per-type LDS arrays, sized by the catalog's T at launch (launch_lds_bytes): ≈32 KB at T = 918, i.e. 5 workgroups
// per CU.  ctok doubles as the Truncate stage's order keys once every type's mask is in registers; key holds the
// CapacityBlockFilter / Truncate prices, the ReservedOfferingFilter winners (win) and, after Truncate, the
// SatisfiesMinValues bitset (minbits).
struct LTypes {
    uint64_t *lv, *ac, *ctok, *win, *minbits;  // live offerings, Available ∧ Compatible w/o capacity type, ct-compatible
    double* key;
    uint8_t *keep, *aux;
    int8_t* pos;  // CapacityBlockFilter offering, then Truncate rank (< M <= 64)
};
__host__ __device__ inline int ltypes_key_len(int T) { return T > KP_MAX_MIN_WORDS ? T : KP_MAX_MIN_WORDS; }
__device__ __forceinline__ LTypes ltypes(char* p, int T) {
    LTypes L;
    L.lv = reinterpret_cast<uint64_t*>(p);
    L.ac = L.lv + T;
    L.ctok = L.ac + T;
    L.key = reinterpret_cast<double*>(L.ctok + T);
    L.win = reinterpret_cast<uint64_t*>(L.key);
    L.minbits = reinterpret_cast<uint64_t*>(L.key);
    L.keep = reinterpret_cast<uint8_t*>(L.key + ltypes_key_len(T));
    L.aux = L.keep + T;
    L.pos = reinterpret_cast<int8_t*>(L.aux + T);
    return L;
}
inline size_t launch_lds_bytes(int T) { return (size_t)(3 * T + ltypes_key_len(T)) * 8 + 3 * (size_t)T; }

__device__ __forceinline__ bool wbit(const uint64_t* w, int off, int v) { return (w[off + (v >> 6)] >> (v & 63)) & 1ull; }

__device__ int bsum(int x, LShared& S) {
    x = (int)wave_reduce32((uint32_t)x, [](uint32_t a, uint32_t b) { return a + b; });
    if ((threadIdx.x & 63) == 0) S.redi[threadIdx.x >> 6] = x;
    __syncthreads();
    int r = 0;
    for (int w = 0; w < NWV; w++) r += S.redi[w];
    __syncthreads();
    return r;
}
__device__ int bmin_i(int x, LShared& S) {
    x = (int)wave_reduce32((uint32_t)x, [](uint32_t a, uint32_t b) { return (int)b < (int)a ? b : a; });
    if ((threadIdx.x & 63) == 0) S.redi[threadIdx.x >> 6] = x;
    __syncthreads();
    int r = S.redi[0];
    for (int w = 1; w < NWV; w++) r = min(r, S.redi[w]);
    __syncthreads();
    return r;
}
__device__ double bmin_d(double x, LShared& S) {
    x = __longlong_as_double((long long)wave_reduce64((uint64_t)__double_as_longlong(x), [](uint64_t a, uint64_t b) {
        return __longlong_as_double((long long)b) < __longlong_as_double((long long)a) ? b : a;
    }));
    if ((threadIdx.x & 63) == 0) S.redd[threadIdx.x >> 6] = x;
    __syncthreads();
    double r = S.redd[0];
    for (int w = 1; w < NWV; w++) r = S.redd[w] < r ? S.redd[w] : r;
    __syncthreads();
    return r;
}

// InstanceType.Requirements vs request: Compatible(AllowUndefinedWellKnownLabels) + Intersects (filter.go:53)
__device__ bool type_compat(const KpLaunch& g, const KlReq& q, int t) {
    for (int j = 0; j < q.n_keys; j++) {
        const KlKey kk = g.keys[q.key_off + j];
        if (kk.flags & KLK_MULTI) {
            const uint64_t m = g.multi_mask[(size_t)kk.mi * g.T + t];
            if (m == 0) {
                const bool dne = (g.dne_mask[(size_t)kk.k * g.TW + (t >> 6)] >> (t & 63)) & 1ull;
                if (dne && !(kk.flags & KLK_DNE_OK)) return false;
                continue;
            }
            if (!(m & g.words[kk.woff])) return false;
        } else {
            const uint32_t v = g.type_val[(size_t)kk.k * g.T + t];
            if (v == VAL_ABSENT) continue;
            if (v == VAL_DNE) {
                if (!(kk.flags & KLK_DNE_OK)) return false;
                continue;
            }
            if (!wbit(g.words, kk.woff, (int)v)) return false;
        }
    }
    for (int j = 0; j < q.n_und; j++) {  // a type label the request leaves undefined must not be an In on a custom key
        const KlKey kk = g.keys[q.und_off + j];
        if (kk.flags & KLK_MULTI) {
            if (g.multi_mask[(size_t)kk.mi * g.T + t]) return false;
        } else {
            const uint32_t v = g.type_val[(size_t)kk.k * g.T + t];
            if (v != VAL_ABSENT && v != VAL_DNE) return false;
        }
    }
    return true;
}

__device__ __forceinline__ bool role_ok(const KpLaunch& g, const KlRole& r, int v) {
    if (v == KL_V_ABSENT) return true;
    if (v == KL_V_DNE) return r.mode != KLR_CONSTRAINED || (r.flags & KLK_DNE_OK);
    if (r.mode == KLR_PASS) return true;
    if (r.mode == KLR_FAIL_IN) return false;
    return wbit(g.words, r.woff, v);
}

__device__ __forceinline__ uint64_t ct_mask(const KpLaunch& g, int o0, uint64_t m, int ct) {
    uint64_t out = 0;
    while (m) {
        const int j = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        if (g.ct_code[o0 + j] == ct) out |= 1ull << j;
    }
    return out;
}

__global__ __launch_bounds__(NT) void launch_kernel(KpLaunch g) {
    __shared__ LShared S;
    extern __shared__ __attribute__((aligned(16))) char ldyn[];
    const int i = blockIdx.x, tid = threadIdx.x, T = g.T, M = g.M;
    const LTypes L = ltypes(ldyn, T);
    const KlReq q = g.req[i];
    const int64_t* rq = g.requests + (size_t)i * g.R;
    int32_t* hdr = g.out_hdr + (size_t)i * KL_HDR;
    int rejected[KP_N_FILTERS] = {0, 0, 0, 0, 0, 0};

    // ---- CompatibleAvailableFilter (filter.go:51-64) ----
    int n = 0;
    for (int t = tid; t < T; t += NT) {
        const int o0 = g.off_begin[t], no = g.off_begin[t + 1] - o0;
        uint64_t cmn = 0, ctok = 0, am = 0;
        for (int j = 0; j < no; j++) {
            const int o = o0 + j;
            bool ok = true;
#pragma unroll
            for (int r = 0; r < KL_ROLES; r++)
                if (r != KL_ROLE_CT) ok = ok && role_ok(g, q.role[r], g.off_val[(size_t)r * (g.off_begin[T]) + o]);
            if (ok) cmn |= 1ull << j;
            if (role_ok(g, q.role[KL_ROLE_CT], g.off_val[(size_t)KL_ROLE_CT * g.off_begin[T] + o])) ctok |= 1ull << j;
            if (g.off_avail[o]) am |= 1ull << j;
        }
        const uint64_t lv = no >= 64 ? ~0ull : ((1ull << no) - 1);
        L.lv[t] = lv;
        L.ac[t] = am & cmn;
        L.ctok[t] = ctok;
        bool keep = (lv & cmn & ctok & am) != 0;
        if (keep) {
            for (int r = 0; r < g.R && keep; r++) keep = !(rq[r] != 0 && rq[r] > g.alloc[(size_t)r * T + t]);
        }
        keep = keep && type_compat(g, q, t);
        L.keep[t] = keep;
        n += keep;
    }
    n = bsum(n, S);
    rejected[0] = T - n;
    int failed = n == 0 ? KP_FILTER_COMPATIBLE_AVAILABLE : -1;

    const bool reserved = q.ct_has[KP_CT_RESERVED] != 0;
    // ---- CapacityReservationTypeFilter (filter.go:83-119) ----
    if (failed < 0 && reserved) {
        double c0 = DBL_MAX, c1 = DBL_MAX;
        for (int t = tid; t < T; t += NT) {
            uint8_t mem = 0;
            if (L.keep[t]) {
                const int o0 = g.off_begin[t];
                uint64_t m = L.lv[t] & L.ac[t] & L.ctok[t];
                while (m) {
                    const int j = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const int o = o0 + j;
                    if (g.ct_code[o] != KP_CT_RESERVED) continue;
                    const int p = g.rt_code[o];
                    const double pr = g.off_price[o];
                    if (p == 0) {
                        mem |= 1;
                        c0 = pr < c0 ? pr : c0;
                    } else if (p == 1) {
                        mem |= 2;
                        c1 = pr < c1 ? pr : c1;
                    }
                }
            }
            L.aux[t] = mem;
        }
        c0 = bmin_d(c0, S);
        c1 = bmin_d(c1, S);
        const int sel = (c1 < c0) ? 1 : 0;  // lo.MinBy: cheaper partition, ties to default (priority 0)
        int cnt = 0;
        for (int t = tid; t < T; t += NT) cnt += L.keep[t] && ((L.aux[t] >> sel) & 1);
        cnt = bsum(cnt, S);
        if (cnt > 0) {
            for (int t = tid; t < T; t += NT) {
                if (!L.keep[t]) continue;
                if ((L.aux[t] >> sel) & 1) {
                    const int o0 = g.off_begin[t];
                    uint64_t m = L.lv[t], nl = 0;
                    while (m) {
                        const int j = __ffsll((unsigned long long)m) - 1;
                        m &= m - 1;
                        if (g.ct_code[o0 + j] == KP_CT_RESERVED && g.rt_code[o0 + j] == sel) nl |= 1ull << j;
                    }
                    L.lv[t] = nl;
                } else {
                    L.keep[t] = 0;
                }
            }
            rejected[1] = n - cnt;
            n = cnt;
        }
        __syncthreads();
    }
    // ---- CapacityBlockFilter (filter.go:173-221) ----
    if (failed < 0 && reserved) {
        // shouldFilter: the first offering (type order, then offering order) that carries the reservation-type key decides
        int first = INT32_MAX;
        for (int t = tid; t < T; t += NT) {
            uint8_t code = 0;
            if (L.keep[t]) {
                const int o0 = g.off_begin[t];
                uint64_t m = L.lv[t];
                while (m) {
                    const int j = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    if (g.off_val[(size_t)KL_ROLE_RESVTYPE * g.off_begin[T] + o0 + j] != KL_V_ABSENT) {
                        code = g.rt_code[o0 + j] == 1 ? 2 : 1;
                        break;
                    }
                }
            }
            L.aux[t] = code;
            if (code) first = min(first, t);
        }
        first = bmin_i(first, S);
        if (first != INT32_MAX && L.aux[first] == 2) {
            double best = DBL_MAX;
            for (int t = tid; t < T; t += NT) {
                L.key[t] = DBL_MAX;
                L.pos[t] = -1;
                if (!L.keep[t]) continue;
                const int o0 = g.off_begin[t];
                uint64_t m = L.lv[t];
                int sj = -1;
                double sp = 0.0;
                while (m) {
                    const int j = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const int o = o0 + j;
                    if (g.ct_code[o] != KP_CT_RESERVED || g.rt_code[o] != 1) continue;
                    if (sj < 0 || sp > g.off_price[o]) {
                        sj = j;
                        sp = g.off_price[o];
                    }
                }
                if (sj >= 0) {
                    L.key[t] = sp;
                    L.pos[t] = (int8_t)sj;
                    best = sp < best ? sp : best;
                }
            }
            best = bmin_d(best, S);
            int win = INT32_MAX;
            for (int t = tid; t < T; t += NT)
                if (L.pos[t] >= 0 && L.key[t] == best) win = min(win, t);
            win = bmin_i(win, S);
            for (int t = tid; t < T; t += NT) {
                if (t == win) L.lv[t] = 1ull << L.pos[t];
                else L.keep[t] = 0;
            }
            rejected[2] = n - 1;
            n = 1;
            __syncthreads();
        }
    }
    // ---- ReservedOfferingFilter (filter.go:240-270) ----
    if (failed < 0 && reserved) {
        int cnt = 0;
        for (int t = tid; t < T; t += NT) {
            L.win[t] = 0;
            if (!L.keep[t]) continue;
            const int o0 = g.off_begin[t];
            uint64_t cand = L.lv[t] & L.ac[t] & L.ctok[t] & ct_mask(g, o0, L.lv[t], KP_CT_RESERVED);
            uint64_t m = cand, win = 0;
            while (m) {  // per zone: the first offering with the greatest ReservationCapacity
                const int j = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const int z = g.off_val[(size_t)KL_ROLE_ZONE * g.off_begin[T] + o0 + j];
                const int cj = g.off_rcap[o0 + j];
                bool best = true;
                uint64_t m2 = cand;
                while (m2 && best) {
                    const int j2 = __ffsll((unsigned long long)m2) - 1;
                    m2 &= m2 - 1;
                    if (j2 == j || g.off_val[(size_t)KL_ROLE_ZONE * g.off_begin[T] + o0 + j2] != z) continue;
                    const int c2 = g.off_rcap[o0 + j2];
                    if (c2 > cj || (c2 == cj && j2 < j)) best = false;
                }
                if (best) win |= 1ull << j;
            }
            L.win[t] = win;
            cnt += win != 0;
        }
        cnt = bsum(cnt, S);
        if (cnt > 0) {
            for (int t = tid; t < T; t += NT) {
                if (!L.keep[t]) continue;
                if (L.win[t]) L.lv[t] = L.win[t];
                else L.keep[t] = 0;
            }
            rejected[3] = n - cnt;
            n = cnt;
        }
        __syncthreads();
    }
    // ---- ExoticInstanceTypeFilter (filter.go:289-318) ----
    if (failed < 0 && !q.has_min) {
        int cnt = 0;
        for (int t = tid; t < T; t += NT) cnt += L.keep[t] && !g.exotic[t];
        cnt = bsum(cnt, S);
        if (cnt > 0) {
            for (int t = tid; t < T; t += NT)
                if (g.exotic[t]) L.keep[t] = 0;
            rejected[4] = n - cnt;
            n = cnt;
        }
        __syncthreads();
    }
    // ---- SpotInstanceFilter (filter.go:339-386) ----
    if (failed < 0 && !q.has_min && q.ct_has[KP_CT_ON_DEMAND] && q.ct_has[KP_CT_SPOT]) {
        double cod = DBL_MAX;
        int has_od = 0, has_spot = 0;
        for (int t = tid; t < T; t += NT) {
            if (!L.keep[t]) continue;
            const int o0 = g.off_begin[t];
            uint64_t m = L.lv[t] & L.ac[t] & L.ctok[t];
            while (m) {
                const int j = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const int ct = g.ct_code[o0 + j];
                if (ct == KP_CT_ON_DEMAND) {
                    has_od = 1;
                    cod = g.off_price[o0 + j] < cod ? g.off_price[o0 + j] : cod;
                } else if (ct == KP_CT_SPOT) {
                    has_spot = 1;
                }
            }
        }
        cod = bmin_d(cod, S);
        has_od = bsum(has_od, S);
        has_spot = bsum(has_spot, S);
        if (has_od && has_spot) {
            int cnt = 0;
            for (int t = tid; t < T; t += NT) {
                if (!L.keep[t]) continue;
                const int o0 = g.off_begin[t];
                uint64_t m = L.lv[t] & L.ac[t] & L.ctok[t];
                bool keep = true, spot = false, cheap = false, resv = false;
                while (m) {
                    const int j = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const int ct = g.ct_code[o0 + j];
                    if (ct == KP_CT_RESERVED) resv = true;
                    if (ct == KP_CT_SPOT) {
                        spot = true;
                        if (g.off_price[o0 + j] <= cod) cheap = true;
                    }
                }
                keep = resv || cheap || !spot;
                L.keep[t] = keep;
                cnt += keep;
            }
            cnt = bsum(cnt, S);
            rejected[5] = n - cnt;
            n = cnt;
            if (n == 0) failed = KP_FILTER_SPOT;
        }
    }

    // ---- Truncate: OrderByPrice (cheapest Available().Compatible(reqs), MaxFloat64 if none, ties by name) ----
    int status = failed >= 0 ? KP_E_INSUFFICIENT_CAPACITY : KP_OK;
    int ct_sel = KP_CT_ON_DEMAND, n_types = 0, n_over = 0;
    if (failed < 0) {
        // compact the kept types: L.key[u] = cheapest compatible available price, ordk[u] = name_rank << 32 | t
        // (order of u is irrelevant: the rank below is a pure count over the (price, name, index) order)
        constexpr int PER = (KP_MAX_TYPES + NT - 1) / NT;
        if (tid == 0) S.ncomp = 0;
        double pk[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int t = tid + k * NT;
            pk[k] = -1.0;  // not kept
            if (t >= T || !L.keep[t]) continue;
            const int o0 = g.off_begin[t];
            uint64_t m = L.lv[t] & L.ac[t] & L.ctok[t];
            double p = DBL_MAX;
            while (m) {
                const int j = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                p = g.off_price[o0 + j] < p ? g.off_price[o0 + j] : p;
            }
            pk[k] = p;
        }
        __syncthreads();  // every ctok read is done: ctok becomes the order keys
        uint64_t* const ordk = L.ctok;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int t = tid + k * NT;
            if (pk[k] < 0.0) continue;
            const int u = atomicAdd(&S.ncomp, 1);
            L.key[u] = pk[k];
            ordk[u] = ((uint64_t)g.name_rank[t] << 32) | (uint32_t)t;
        }
        __syncthreads();
        const int nc = S.ncomp;
        int my_t[PER], my_r[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            my_t[k] = -1;
            my_r[k] = M;
            const int u = tid + k * NT;
            if (u >= nc) continue;
            const double kt = L.key[u];
            const uint64_t pt = ordk[u];
            int rank = 0;
            for (int v = 0; v < nc && rank < M; v++) {
                const double kv = L.key[v];
                rank += (kv < kt) || (kv == kt && ordk[v] < pt);
            }
            my_t[k] = (int)(uint32_t)pt;
            my_r[k] = rank;
        }
        for (int t = tid; t < T; t += NT) L.pos[t] = -1;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PER; k++)
            if (my_t[k] >= 0 && my_r[k] < M) {
                L.pos[my_t[k]] = (int8_t)my_r[k];
                g.out_types[(size_t)i * M + my_r[k]] = my_t[k];
            }
        n_types = n < M ? n : M;
        __syncthreads();
        // SatisfiesMinValues over the truncated list (monotone in the prefix, so the full list decides)
        for (int mk = 0; mk < q.n_min && status == KP_OK; mk++) {
            const KlMinKey mkey = g.mins[q.min_off + mk];
            for (int w = tid; w < KP_MAX_MIN_WORDS; w += NT) L.minbits[w] = 0;
            __syncthreads();
            for (int t = tid; t < T; t += NT) {
                if (L.pos[t] < 0) continue;
                if (mkey.mi >= 0) {
                    const uint64_t mm = g.multi_mask[(size_t)mkey.mi * T + t];
                    if (mm) atomicOr((unsigned long long*)&L.minbits[0], (unsigned long long)mm);
                } else {
                    const uint32_t v = g.type_val[(size_t)mkey.k * T + t];
                    if (v != VAL_ABSENT && v != VAL_DNE)
                        atomicOr((unsigned long long*)&L.minbits[v >> 6], 1ull << (v & 63));
                }
            }
            __syncthreads();
            int c = 0;
            for (int w = tid; w < KP_MAX_MIN_WORDS; w += NT) c += __popcll(L.minbits[w]);
            c = bsum(c, S);
            if (c < mkey.minv) status = KP_E_CREATE;
        }
        // getCapacityType (instance.go:532-546)
        if (status == KP_OK) {
            const int order[2] = {KP_CT_RESERVED, KP_CT_SPOT};
            for (int oi = 0; oi < 2; oi++) {
                const int ct = order[oi];
                if (!q.ct_has[ct]) continue;
                int any = 0;
                for (int t = tid; t < T; t += NT) {
                    if (L.pos[t] < 0) continue;
                    const int o0 = g.off_begin[t];
                    any |= (L.lv[t] & L.ac[t] & ct_mask(g, o0, L.lv[t], ct)) != 0;
                }
                any = bsum(any, S);
                if (any) {
                    ct_sel = ct;
                    break;
                }
            }
            // getOverrides: Available ∧ Compatible(reqs with capacity-type := In[ct_sel]), per kept type in price order
            for (int t = tid; t < T; t += NT) {
                if (L.pos[t] < 0) continue;
                const int o0 = g.off_begin[t];
                uint64_t m = L.lv[t] & L.ac[t] & ct_mask(g, o0, L.lv[t], ct_sel);
                g.out_over[(size_t)i * M + L.pos[t]] = m;  // the host expands bit j to offering row o0 + j
                n_over += __popcll(m);
            }
            n_over = bsum(n_over, S);
        }
    }
    if (tid == 0) {
        hdr[0] = status;
        hdr[1] = failed;
        hdr[2] = ct_sel;
        hdr[3] = status == KP_OK ? n_types : 0;
        hdr[4] = n_over;
        hdr[5] = failed >= 0 ? 0 : n;
        hdr[6] = hdr[7] = 0;
        for (int f = 0; f < KP_N_FILTERS; f++) hdr[8 + f] = rejected[f];
    }
}

}  // namespace

hipError_t kp_launch_select_kernel(const KpLaunch& g, hipStream_t s) {
    if (g.L <= 0) return hipSuccess;
    hipLaunchKernelGGL(launch_kernel, dim3(g.L), dim3(NT), launch_lds_bytes(g.T), s, g);
    return hipGetLastError();
}
