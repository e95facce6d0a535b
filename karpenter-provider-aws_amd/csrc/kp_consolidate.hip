// kp_consolidate.hip — consolidation probes on gfx950: one wave per SimulateScheduling + computeConsolidation.
//
// Reference semantics ([core] sigs.k8s.io/karpenter pkg/controllers/disruption, recalled):
//   SimulateScheduling (helpers.go): state nodes minus the candidates, pods = pending + candidates' reschedulable
//     pods, NewScheduler (NodePool limits recomputed without the candidates), Solve, TruncateInstanceTypes(60); a pod
//     placed on an uninitialized node is an error.
//   computeConsolidation (consolidation.go): not all non-pending pods scheduled → NONE; no new NodeClaim → DELETE;
//     more than one → NONE; else the NodeClaim's options OrderByPrice'd, spot-to-spot gate (computeSpotToSpotConsolidation:
//     feature gate, ≥ 15 cheaper types for one candidate, the 15 cheapest kept), otherwise
//     RemoveInstanceTypeOptionsByPriceAndMinValues(WorstLaunchPrice < Σ candidate prices) and capacity-type
//     narrowed to spot when both spot and on-demand remain.
//   multinodeconsolidation.go: filterOutSameInstanceType on a REPLACE (the search's validity test).
//
// Per probe the wave keeps: an exclusion bitmap of its candidates and a modified-node bitmap (LDS), the requests it
// added to existing nodes (global delta slab, read past L1), the queue as a ring in global memory with a 64-entry
// register window, and at most one in-flight NodeClaim (requirements digest, options, requests) in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cfloat>

#include "kp_cons.h"
#include "kp_device.h"
#include "kp_eval.h"
#include "kp_layout.h"

namespace {

struct ConsShared {
    ClassCache CC;
    WaveScratch ws;
    Roles roles;
    int64_t nc_req[KP_MAX_R];
    int64_t st[CS_COUNT];
    uint64_t mro[KP_RO_W];  // RESV: the reserved-offering rows compatible with the probe's NodeClaim (its finalisation)
    uint64_t born;          // TOPO: the probe's late topology identities created so far (ProbeTopo::born)
};

__device__ __forceinline__ int32_t ld32(const int32_t* p) {
    return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld64u(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wave-uniform values read from LDS: the compiler cannot prove them uniform, and a branch on them would make the
// pod loop's control flow divergent (exec-mask save/restore around every chunk test); readfirstlane keeps them scalar.
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}
__device__ __forceinline__ int wave_sum_i32(int x) {
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ double wave_min_f64(double x) {
    for (int o = 32; o >= 1; o >>= 1) {
        const double y = __shfl_xor(x, o);
        x = y < x ? y : x;
    }
    return x;
}

// types whose Capacity exceeds the probe's remaining NodePool limits (filterByRemainingResources)
__device__ inline uint64_t limit_filter_rem(const KpDev& d, int j, uint64_t o, const int64_t* rem, int lane) {
    bool any_limit = false;
    for (int r = 0; r < d.R; r++) any_limit |= d.limit_set[(size_t)j * d.R + r] != 0;
    if (!any_limit) return o;
    uint64_t out = 0;
    for (int w = 0; w < d.TW; w++) {
        const uint64_t cw = rl64(o, w);
        if (!cw) continue;
        const int t = w * 64 + lane;
        bool keep = (cw >> lane) & 1ull;
        if (keep) {
            for (int r = 0; r < d.R; r++)
                if (d.limit_set[(size_t)j * d.R + r] && d.cap[(size_t)r * d.T + t] > rem[j * d.R + r]) keep = false;
        }
        const uint64_t nb = ballot(keep);
        if (lane == w) out = nb;
    }
    return out;
}

// Offerings.Available().WorstLaunchPrice(reqs) over the admissible slots m and reserved offerings rm (bits of ResvTab
// word rw) of type t: reserved, then spot, then on-demand; the most expensive offering of the first capacity type present.
__device__ inline double worst_launch_price(const KpDev& d, const KpCons& k, int t, uint64_t m, uint64_t rm = 0, int rw = 0) {
    if (rm) {
        double mx = 0.0;
        for (uint64_t x = rm; x; x &= x - 1) {
            const double p = d.ro_price[rw * 64 + __ffsll((unsigned long long)x) - 1];
            mx = p > mx ? p : mx;
        }
        return mx;
    }
    const uint64_t ms = m & k.spot_slots;
    uint64_t mm = ms ? ms : (m & k.od_slots);
    if (!mm) return DBL_MAX;
    double mx = 0.0;
    bool first = true;
    while (mm) {
        const int s = __ffsll((unsigned long long)mm) - 1;
        mm &= mm - 1;
        const double p = d.slot_price[(size_t)t * KP_MAX_SLOTS + s];
        if (first || p > mx) mx = p;
        first = false;
    }
    return mx;
}

// minValues over an ordered option list held one type per lane (lane i = the i-th cheapest, lanes in `m` kept):
// the distinct values of single-valued catalog key k (a type without the label contributes none, like
// Requirements.Get(k).Values()).  Returns the lanes holding a first occurrence, in lane order.
__device__ inline uint64_t first_values(const KpDev& d, int k, int my_t, uint64_t m, int lane) {
    const int kc = d.kcat[k];
    int v = -1;
    if (((m >> lane) & 1ull) && kc >= 0 && my_t >= 0) {
        const uint16_t x = d.type_val[(size_t)kc * d.T + my_t];
        if (x < VAL_ABSENT) v = x;
    }
    bool first = v >= 0;
    for (int j = 0; j < 63; j++) {
        const int vj = __shfl(v, j);
        if (j < lane && vj == v) first = false;
    }
    return ballot(first);
}

// The same for a multi-valued catalog key (zone, capacity-type, ...: <= 64 values, one mask per type): lane i gets the
// number of distinct values over the kept lanes <= i (an inclusive prefix OR of the masks).
__device__ inline int multi_values_upto(const KpDev& d, int k, int my_t, uint64_t m, int lane) {
    uint64_t v = (((m >> lane) & 1ull) && my_t >= 0) ? d.multi_mask[(size_t)d.kmulti[k] * d.T + my_t] : 0ull;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(v >> 32), o) << 32) |
                           (uint32_t)__shfl_up((int)(uint32_t)v, o);
        if (lane >= o) v |= y;
    }
    return __popcll(v);
}

// InstanceTypes.SatisfiesMinValues over the kept lanes m of NodeClaim template j's minValues keys (header nch):
// *need = minNeededInstanceTypes, the shortest kept prefix that satisfies every key.
__device__ inline bool min_values_ok(const KpDev& d, const ReqHdr* nch, int j, int my_t, uint64_t m, int lane, int* need) {
    const int* mk = d.min_keys + (size_t)j * KP_MAX_CLASS_KEYS;
    int nd = 0;
    for (int q = 0; q < KP_MAX_CLASS_KEYS; q++) {
        const int k = mk[q];
        if (k < 0) break;
        const ReqHdr h = nch[k];
        if (!(h.flags & RF_MIN) || h.minv <= 0) continue;
        int L;
        if (d.kmulti[k] >= 0) {
            const int upto = multi_values_upto(d, k, my_t, m, lane);
            const uint64_t reach = ballot(upto >= h.minv);
            if (!reach) return false;
            L = __ffsll((unsigned long long)reach) - 1;
        } else {
            const uint64_t f = first_values(d, k, my_t, m, lane);
            if (__popcll(f) < h.minv) return false;
            // the kept lane at which the count reaches minv, as a position in the kept list
            uint64_t x = f;
            for (int i = 1; i < h.minv; i++) x &= x - 1;
            L = __ffsll((unsigned long long)x) - 1;
        }
        const int pos = __popcll(m & ((L >= 63) ? ~0ull : ((2ull << L) - 1)));
        nd = pos > nd ? pos : nd;
    }
    if (need) *need = nd;
    return true;
}

// MIN_VALUES_POLICY=BestEffort: the Add's relaxed minValues into the probe's NodeClaim digest (after its class keys).
__device__ inline void commit_min_relax_lds(ReqHdr* nch, const WaveScratch& ws, int lane) {
    if (lane < ws.n_minrel) nch[ws.minrel_k[lane]].minv = ws.minrel_v[lane];
    __syncthreads();
}

}  // namespace

// NodeClaim.Add's commit of offeringsToReserve (fallback mode): newly held reservations take one unit of capacity,
// those no longer held are released (ReservationManager.Reserve / Release).  Lane r: word r of the held set (old), the
// Add's set in ws.minbits; returns the new word.
__device__ inline uint64_t commit_held(int32_t* rcap, uint64_t old, const WaveScratch& ws, int ridw, int lane) {
    if (lane >= ridw) return 0ull;
    const uint64_t nw = ws.minbits[lane];
    for (uint64_t x = nw & ~old; x; x &= x - 1) rcap[lane * 64 + __ffsll((unsigned long long)x) - 1]--;
    for (uint64_t x = old & ~nw; x; x &= x - 1) rcap[lane * 64 + __ffsll((unsigned long long)x) - 1]++;
    return nw;
}

// FULL = false: the fast variant handles probes whose pods all fit existing nodes (no NodeClaim code, a small register
// footprint); a probe that needs a NodeClaim is handed to the FULL variant through k.retry.
// RESV (FULL only): the catalog has reserved offerings — NodeClaim.Add runs the reservation step in
// ReservedOfferingModeFallback (SimulateScheduling never fails an Add for want of a reservation), the in-flight
// NodeClaim's held IDs take / release the probe's capacities, FinalizeScheduling adds reservation-id In [held], and
// OrderByPrice / WorstLaunchPrice see the reserved offerings.
// TOPO: the cluster's pods carry topology terms — each probe keeps its own domain counts (ProbeTopo: the prepared base of
// every bound pod minus the pods it reschedules); pods of constrained classes run ExistingNode.Add's
// Topology.AddRequirements on each candidate node (first-fit over the nodes that pass, never memoised: counts move) and
// NodeClaim.Add's on the in-flight NodeClaim (hostname row E) and on templates (a fresh hostname, count 0); every
// placement of a counted class is recorded.
// NA (fast variant only): the number of active axes, fixed at compile time so that the window intake's per-axis tests
// and prefix sums unroll without runtime guards (0: read from d.n_active).
// MUT (FULL only): the pass has probes that reschedule a mutator's pod (KpCons::mut): such a probe runs serially over its
// queue and applies ExistingNode.Add's requirement merge to its own copies of the nodes it changes (see KpCons).
#define AXL(ai) _Pragma("unroll") for (int ai = 0; ai < (NA > 0 ? NA : KP_LDS_AXES); ai++) if (NA > 0 || ai < A)
// DevT / ConsT: KpDev / KpCons by value (the fast variant: its kernel arguments) or const references to the FULL
// variant's device copies — a by-value copy of those, indexed dynamically (active_axes ...), went to scratch per lane
// (1.3 KB per lane, 87 MB of scratch writes per replace-leg launch).
template <bool FULL, bool RESV = false, bool TOPO = false, int NA = 0, bool MUT = false, class DevT = KpDev,
          class ConsT = KpCons>
__device__ __forceinline__ void consolidate_body(DevT d, ConsT k) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    ConsShared& S = *reinterpret_cast<ConsShared*>(smem);
    ReqHdr* nch = reinterpret_cast<ReqHdr*>(smem + k.off_hdr);
    uint64_t* ncw = reinterpret_cast<uint64_t*>(smem + k.off_words);
    int64_t* rem = reinterpret_cast<int64_t*>(smem + k.off_rem);
    uint64_t* excl = reinterpret_cast<uint64_t*>(smem + k.off_excl);
    uint64_t* modb = reinterpret_cast<uint64_t*>(smem + k.off_mod);
    uint64_t* initb = reinterpret_cast<uint64_t*>(smem + k.off_init);
    uint64_t* xtc = reinterpret_cast<uint64_t*>(smem + k.off_xtc);  // XT column of the cached chunk, by class
    int64_t* cmax = reinterpret_cast<int64_t*>(smem + k.off_cmax);  // [EW][KP_LDS_AXES] chunk headroom upper bounds
    uint64_t* mutn = reinterpret_cast<uint64_t*>(smem + k.off_mutn);  // MUT: nodes whose requirements the probe changed
    const int lane = threadIdx.x;
    ProbeTopo P{};
    if (TOPO) {
        P.cnt = k.pt_cnt + (size_t)blockIdx.x * k.G * 64;
        P.known = k.pt_known + (size_t)blockIdx.x * k.G;
        P.touched = reinterpret_cast<uint64_t*>(smem + k.off_touch);
        P.hd = k.pt_hd + (size_t)blockIdx.x * k.HG * (d.E + 1);
        P.hmod = reinterpret_cast<uint64_t*>(smem + k.off_hmod);
        P.dgk = k.pt_dgk;
        P.hpos = reinterpret_cast<int32_t*>(smem + k.off_hpos);
        P.ha = k.tg_ha;
        P.born = &S.born;
        P.excl = excl;
        P.E = d.E;
        P.HG = k.HG;
    }
    // input classes / shapes of the pods (pod_cls0 when preferences can relax: a Solve execute rewrites pod_cls)
    const int32_t* const pcls = d.pod_cls0 ? d.pod_cls0 : d.pod_cls;
    const int32_t* const pshape = d.pod_shape0 ? d.pod_shape0 : d.pod_shape;
    const int wid = blockIdx.x;
    const int E = d.E, EW = d.EW, A = d.n_active, R = d.R, K = d.K, TW = d.TW, T = d.T, NT = d.NT;
    const int cap = k.ring_cap;
    int32_t* ring = k.ring + (size_t)wid * cap;
    int32_t* rlast = k.ring_last + (size_t)wid * cap;
    int32_t* rcls = k.relax ? k.ring_cls + (size_t)wid * cap : nullptr;
    int32_t* rshape = k.relax ? k.ring_shape + (size_t)wid * cap : nullptr;
    int64_t* delta = k.delta + (size_t)wid * A * (E > 0 ? E : 1);
    uint64_t* pbits = k.pbits + (size_t)wid * k.PW;
    int32_t* const ov_slot = MUT ? k.ov_slot + (size_t)wid * (E > 0 ? E : 1) : nullptr;
    ReqHdr* const ov_hdr = MUT ? k.ov_hdr + (size_t)wid * k.ov_cap * K : nullptr;
    uint64_t* const ov_words = MUT ? k.ov_words + (size_t)wid * k.ov_cap * d.DW : nullptr;

    if (lane < 5) {
        const int rk = lane == 0 ? d.key_zone : lane == 1 ? d.key_ct : lane == 2 ? d.key_zoneid : lane == 3 ? d.key_resvid : d.key_resvtype;
        S.roles.key[lane] = rk;
        S.roles.woff[lane] = rk >= 0 ? d.woff[rk] : 0;
        S.roles.nw[lane] = rk >= 0 ? d.nw[rk] : 0;
    }
    if (lane == 0) S.CC.cls = -1;
    if (lane < CS_COUNT) S.st[lane] = 0;
    for (int w = lane; w < EW; w += 64) initb[w] = k.init_bits[w];
    __syncthreads();
    EvalEnv Ev;
    Ev.alloc = k.alloc_act;
    Ev.astride = k.astride;
    Ev.avail = d.avail_zc;
    Ev.multi16 = nullptr;
    Ev.slot_zone = d.slot_zone;
    Ev.slot_ct = d.slot_ct;
    Ev.slot_zoneid = d.slot_zoneid;
    Ev.roles = &S.roles;
    {
        uint64_t mmask = 0;  // templates whose requirements carry minValues
        for (int j = 0; j < d.NT; j++)
            if (d.min_keys[(size_t)j * KP_MAX_CLASS_KEYS] >= 0) mmask |= 1ull << j;
        Ev.min_tmpl_mask = mmask;
    }
    Ev.ro = RESV ? d.ro : nullptr;
    Ev.type_ro = RESV ? d.type_ro : nullptr;
    int32_t* const rcap = RESV ? reinterpret_cast<int32_t*>(smem + k.off_rcap) : nullptr;  // [nrid]
    Ev.rcap = rcap;
    Ev.resv_on = RESV ? d.resv_on : 0;  // disruption simulations: ReservedOfferingModeFallback (STRICT = false below)
    Ev.pt = TOPO ? &P : nullptr;
    Ev.snap = nullptr;

    for (int it = 0;; it++) {
        int probe = 0;
        if (!FULL) {  // static stride: a shared work counter serialises in L2 at thousands of probes
            const int nm = k.mode == KP_CONSOLIDATE_BOTH ? k.n_multi : 0;
            const int G = (int)gridDim.x;
            if (nm > 0 && G >= 2 * nm) {
                // the pass waits for its longest probes, the multi-node prefixes: their workers take nothing else, the
                // single-node probes stride over the other workers
                if (wid < nm) probe = it == 0 ? wid : k.n_probes;
                else probe = nm + (wid - nm) + it * (G - nm);
            } else {
                probe = wid + it * G;
            }
        } else {
            if (lane == 0) {
                if (k.no_fast == 1) {
                    probe = atomicAdd(&k.next_probe[0], 1);
                } else {
                    const int i = atomicAdd(&k.next_probe[1], 1);
                    probe = i < ld32(&k.next_probe[2]) ? k.retry[i] : k.n_probes;
                }
            }
            probe = __builtin_amdgcn_readfirstlane(__shfl(probe, 0));
        }
        if (probe >= k.n_probes) break;
        // work slot → probe: multi-node prefixes are taken longest first (the pass waits for its longest probe, so it
        // must start first); with KP_CONSOLIDATE_BOTH the single-node probes follow them in the same launch
        const int nmul = k.mode == KP_CONSOLIDATE_MULTI ? k.n_probes : (k.mode == KP_CONSOLIDATE_BOTH ? k.n_multi : 0);
        const bool single = probe >= nmul;
        const int oi = single ? probe : nmul - 1 - probe;  // output index
        const int gp = single ? (k.mode == KP_CONSOLIDATE_BOTH ? k.sprobe0 + probe - nmul : k.probe0 + probe) : k.probe0 + oi;
        const int c0 = single ? gp : 0, c1 = single ? gp + 1 : gp + 2;
        int64_t st_pops = 0, st_nodes = 0, st_nc = 0, st_tmpl = 0, st_words = 0, st_placed = 0, st_loads = 0, st_hits = 0;
        int64_t st_skips = 0, st_relax = 0;
        long long pf_load = 0, pf_prep = 0, pf_nodes = 0, pf_visits = 0;  // KPSIM_PROFILE: fast-path stages
        long long pf_many = 0, pf_iters = 0, pf_miss_cyc = 0, pf_miss = 0;
        long long cy_build = 0, cy_scan = 0, cy_nc = 0, cy_dec = 0;
        const bool prof = k.profile != 0;
        const long long cy0 = prof ? __builtin_amdgcn_s_memtime() : 0;

        // ---- probe state: excluded candidates, modified nodes, NodePool limits + candidate capacity ----
        for (int w = lane; w < EW; w += 64) {
            excl[w] = 0;
            modb[w] = 0;
            if (MUT) mutn[w] = 0;
        }
        // a MUT probe reschedules a mutator's pod: the fast variants hand it over, the MUT variant runs it serially
        const bool mutp = k.mut && __builtin_amdgcn_readfirstlane(single ? k.mut_s[gp] : k.mut_m[gp]) != 0;
        int n_ov = 0;  // MUT: node digest copies taken by this probe
        for (int i = lane; i < NT * R; i += 64) rem[i] = d.remaining[i];
        if (k.use_cmax)
            for (int i = lane; i < EW * KP_LDS_AXES; i += 64) cmax[i] = k.cmax0[i];
        if (RESV)
            for (int i = lane; i < d.ro_nrid; i += 64) rcap[i] = d.rcap0[i];
        __syncthreads();
        for (int c = c0 + lane; c < c1; c += 64) {
            const int node = k.cand_i[c * 4 + 0];
            atomicOr((unsigned long long*)&excl[node >> 6], 1ull << (node & 63));
        }
        if (TOPO) {
            // this probe's NewTopology: no row copied yet, no node column of its own; then the pods it reschedules come
            // off the base counts
            for (int w = lane; w < ((k.G + 63) >> 6); w += 64) P.touched[w] = 0;
            for (int w = lane; w < EW; w += 64) P.hmod[w] = 0;
            __syncthreads();
            const int r0 = single ? k.dec_soff[gp] : k.dec_moff[gp], r1 = single ? k.dec_soff[gp + 1] : k.dec_moff[gp + 1];
            for (int r = r0; r < r1; r++) pt_init_row(d, P, k.dec_g[r], k.dec_v + (size_t)r * 64, lane);
            for (int ga = lane; ga < k.n_ha; ga += 64) P.hpos[ga] = k.hpos0[(size_t)(single ? gp : k.n_cand + gp) * k.n_ha + ga];
            if (lane == 0) {
                S.born = k.born_s ? (single ? k.born_s[gp] : k.born_m[gp]) : ~0ull;
                if (d.late_sib) S.CC.cls = -1;  // the class caches route variant groups by this probe's births
            }
        }
        // the probe's candidates are [c0, c1) and their pods one contiguous run of cand_pods (CSR in candidate order)
        const int po0 = k.cand_off[c0], po1 = k.cand_off[c1];
        const int n_np = po1 - po0;
        // getCandidatePrices (Σ in candidate order, as Go adds them), the all-spot test, and the candidates' capacity
        // back into their NodePools' remaining limits; candidates 64 at a time, one per lane, so the probe pays one load
        // latency per 64 candidates, not one per candidate
        double cprice = 0.0;
        bool all_spot = true;
        for (int cb = c0; cb < c1; cb += 64) {
            const int c = cb + lane;
            const bool v = c < c1;
            const double pr = v ? k.cand_price[c] : 0.0;
            const int4 cit = v ? reinterpret_cast<const int4*>(k.cand_i)[c] : make_int4(0, KP_CT_SPOT, 0, -1);
            if (ballot(cit.y != KP_CT_SPOT)) all_spot = false;
            const int nv = c1 - cb < 64 ? c1 - cb : 64;
            const uint32_t plo = (uint32_t)__double2loint(pr), phi = (uint32_t)__double2hiint(pr);
            for (int i = 0; i < nv; i++)
                cprice += __hiloint2double(__builtin_amdgcn_readlane((int)phi, i), __builtin_amdgcn_readlane((int)plo, i));
            if (cit.w >= 0)
                for (int r = 0; r < R; r++)
                    if (d.limit_set[(size_t)cit.w * R + r])
                        atomicAdd((unsigned long long*)&rem[cit.w * R + r], (unsigned long long)k.cand_cap[(size_t)c * R + r]);
        }
        // ---- the probe's pods in queue order ----
        int n = 0;
        if (!single && k.ulist) {
            // multi-node prefix: the call's union list in queue order, filtered to candidates [0, c1) and pending pods
            const int ul = ld32(k.ulen);
            int2 nx = lane < ul ? k.ulist[lane] : make_int2(0, INT32_MAX);
            for (int b = 0; b < ul; b += 64) {
                const int2 e = nx;
                nx = b + 64 + lane < ul ? k.ulist[b + 64 + lane] : make_int2(0, INT32_MAX);
                const bool keep = e.y < c1;
                const uint64_t m = ballot(keep);
                if (keep) {
                    const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
                    ring[pos] = e.x;
                    rlast[pos] = -1;
                }
                n += __popcll(m);
            }
        } else if (k.n_pending == 0 && n_np <= 64) {
            // at most one pod per lane: bitonic sort of (queue position, pod) across the wave
            const int myp = lane < n_np ? k.cand_pods[po0 + lane] : -1;
            uint64_t key = myp >= 0 ? ((uint64_t)(uint32_t)k.rank[myp] << 32) | (uint32_t)myp : ~0ull;
            for (int kk = 2; kk <= 64; kk <<= 1)
                for (int j = kk >> 1; j > 0; j >>= 1) {
                    const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), j) << 32) |
                                       (uint32_t)__shfl_xor((int)(uint32_t)key, j);
                    const bool up = (lane & kk) == 0, lower = (lane & j) == 0;
                    const uint64_t mn = o < key ? o : key, mx = o < key ? key : o;
                    key = (lower == up) ? mn : mx;
                }
            if (lane < n_np) {
                ring[lane] = (int32_t)(uint32_t)key;
                rlast[lane] = -1;
            }
            n = n_np;
        } else {
        // mark queue positions, then scan the bitmap with the pending pods (the next 64 words' loads issued before the
        // current ones are expanded)
        for (int i = po0 + lane; i < po1; i += 64) {
            const int r = k.rank[k.cand_pods[i]];
            __hip_atomic_fetch_or(&pbits[r >> 6], 1ull << (r & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        uint64_t nmine = 0, npend = 0;
        if (lane < k.PW) {
            nmine = ld64u(&pbits[lane]);
            npend = k.n_pending ? k.pend_bits[lane] : 0ull;
        }
        for (int wb = 0; wb < k.PW; wb += 64) {
            const int w = wb + lane;
            const uint64_t mine = nmine, pend = npend;
            nmine = npend = 0;
            if (w + 64 < k.PW) {
                nmine = ld64u(&pbits[w + 64]);
                npend = k.n_pending ? k.pend_bits[w + 64] : 0ull;
            }
            uint64_t x = mine | pend;
            if (!ballot(x != 0)) continue;
            const int cnt = __popcll(x);
            const int v = (int)wave_scan_add32((uint32_t)cnt);
            const int total = __builtin_amdgcn_readlane(v, 63);
            int pos = n + v - cnt;
            while (x) {
                const int b = __ffsll((unsigned long long)x) - 1;
                x &= x - 1;
                const int r = w * 64 + b;
                ring[pos] = d.queue0[r] | (int32_t)(((pend >> b) & 1ull) << 31);
                rlast[pos] = -1;
                pos++;
            }
            if (mine) __hip_atomic_store(&pbits[w], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            n += total;
        }
        st_words += k.PW;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();

        if (prof) cy_build = __builtin_amdgcn_s_memtime() - cy0;
        // ---- Solve: queue with lastLen termination; existing nodes, the in-flight NodeClaim, the templates ----
        int head = 0, count = n, wbase = -64;
        int vpod = -1, vlast = -1, vc = 0, vshape = -1, vpn = -1;
        int64_t vq[KP_LDS_AXES];
#pragma unroll
        for (int ai = 0; ai < KP_LDS_AXES; ai++) vq[ai] = 0;
        auto win_load = [&](int base) {
            wbase = base;
            const int pos = base + lane;
            vpod = -1;
            vlast = -1;
            vc = 0;
            vshape = -1;
            if (pos < head + count) {
                const int slot = pos % cap;
                vpod = ld32(&ring[slot]);
                vlast = ld32(&rlast[slot]);
                if (FULL && !TOPO) vpn = ld32(&k.pnode[(size_t)wid * cap + slot]);
                const int p = vpod & 0x3fffffff;
                if (vpod & 0x40000000) {  // a relaxed entry: its class (| fresh << 31) and shape
                    vc = ld32(&rcls[slot]);
                    vshape = ld32(&rshape[slot]);
                } else {
                    vc = pcls[p];
                    vshape = pshape[p];
                }
#pragma unroll
                for (int ai = 0; ai < KP_LDS_AXES; ai++)
                    vq[ai] = ai < A ? d.pod_req[(size_t)p * R + d.active_axes[ai]] : 0;
            }
        };
        int n_nc = 0, nc_tmpl = -1, prev_shape = -1, xstart = 0, ok_np = 0, nc_nonpend = 0;
        int nc_lc = -1;  // the class whose requirements the in-flight NodeClaim last merged (its Add is then Fits only)
        int relax_at = -1;  // queue position of the last Queue.Push(pod, relaxed): every lastLen pushed before is gone
        bool aborted = !FULL && mutp;  // a MUT probe: the FULL variant's MUT instantiation redoes it
        int cbase = -1, ccls = -1;  // cached node chunk (wave-uniform)
        uint64_t cx = 0;
        // the cached chunk's words of the modified-node bitmap (written back to LDS when the chunk is evicted) and of
        // the initialized-node bitmap: the per-pod commit touches no LDS
        uint64_t cmod = 0, cinit = 0;
        int64_t ch[KP_LDS_AXES], cd[KP_LDS_AXES];
#pragma unroll
        for (int ai = 0; ai < KP_LDS_AXES; ai++) ch[ai] = cd[ai] = 0;
        bool bad = false, stop = false;
        uint64_t nc_opts = 0;
        uint64_t nc_held = 0;  // RESV: lane r: word r of the reservations the in-flight NodeClaim holds
        // Largest headroom of the cached chunk's nodes that are not candidates (lanes past E hold 0): the chunk's entry
        // of the headroom summary when the chunk leaves the registers.
        auto chunk_max = [&](int base, const int64_t (&h)[KP_LDS_AXES], int ai) -> int64_t {
            const bool in = base + lane < E && !((excl[base >> 6] >> lane) & 1ull);
            return wave_max64(in ? h[ai] : INT64_MIN);
        };
        // ExistingNode.Add in scheduling order from node xs (candidates excluded) for a pod of class c requesting q on
        // the active axes: the first node that takes it, or -1.  64-node aligned chunks; the chunk of the last placement
        // stays in registers (effective headroom and this probe's added requests per lane) and becomes the chunk of the
        // returned node.  Other chunks are first filtered 64 at a time (one lane per chunk) by the pod's compatible
        // nodes and the headroom summary, so a pod that fits nowhere skips the cluster without loading it.
        // wide: more requested resource axes than the registers hold (A > KP_LDS_AXES): the axes past KP_LDS_AXES are
        // checked per candidate node from HBM (ex_head minus this probe's delta slab, which holds them as soon as a
        // node takes a pod), and the probe runs the serial queue only (no window pass; the fast variant is not used)
        const bool wide = A > KP_LDS_AXES;
        // serial: no window pass, every pod of the queue scans the existing nodes itself (wide probes; MUT probes, whose
        // node compatibility changes as pods land)
        const bool serial = wide || (MUT && mutp);
        // MUT: the requirements digest of node j as this probe sees it (its copy once a merge changed it)
        auto node_digest = [&](int j, const ReqHdr*& h, const uint64_t*& w) {
            h = d.ex_hdr + (size_t)j * K;
            w = d.ex_words + (size_t)j * d.DW;
            if (MUT && mutp && ((uni64(mutn[j >> 6]) >> (j & 63)) & 1ull)) {
                const int s = __builtin_amdgcn_readfirstlane(ld32(&ov_slot[j]));
                h = ov_hdr + (size_t)s * K;
                w = ov_words + (size_t)s * d.DW;
            }
        };
        // MUT: class c's compatible nodes of chunk w (xw from XT) with the nodes this probe changed re-evaluated against
        // their copies: taints tolerated ∧ static fit ∧ Requirements.Compatible(node copy, class)
        auto mut_patch = [&](int c, int w, uint64_t xw) -> uint64_t {
            if (!(MUT && mutp)) return xw;
            const uint64_t mw = uni64(mutn[w] & ~excl[w]);
            if (!mw) return xw;
            bool ok = false;
            if ((mw >> lane) & 1ull) {
                const int j = w * 64 + lane;
                const int s = ld32(&ov_slot[j]);
                ok = d.ex_static[j] && ((d.ex_tol[(size_t)c * EW + w] >> lane) & 1ull) &&
                     node_compatible(d, ov_hdr + (size_t)s * K, ov_words + (size_t)s * d.DW, c);
            }
            return uni64((xw & ~mw) | ballot(ok));
        };
        // MUT: ExistingNode.Add's requirement merge of a pod of class c placed on node j (nodeRequirements.Add(pod
        // requirements), then .Add(topology requirements): for a topology class ws holds the merged class keys).  The
        // first merge that changes the node copies its digest; a node's labels are single values that a compatible
        // merge keeps, so only a class key the node lacks can change it.
        auto mut_commit = [&](int c, int j, bool from_ws) {
            int s;
            if (!((uni64(mutn[j >> 6]) >> (j & 63)) & 1ull)) {
                bool ch = false;
                for (int i = d.cls_xkoff[c] + lane; i < d.cls_xkoff[c + 1]; i += 64)
                    ch |= !(d.ex_hdr[(size_t)j * K + d.cls_xkeys[i]].flags & RF_DEF);
                if (!ballot(ch)) return;
                s = n_ov++;
                for (int i = lane; i < K; i += 64) ov_hdr[(size_t)s * K + i] = d.ex_hdr[(size_t)j * K + i];
                for (int i = lane; i < d.DW; i += 64) ov_words[(size_t)s * d.DW + i] = d.ex_words[(size_t)j * d.DW + i];
                if (lane == 0) {
                    __hip_atomic_store(&ov_slot[j], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    mutn[j >> 6] |= 1ull << (j & 63);
                }
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // the copy is visible to every lane (past L1)
            } else {
                s = __builtin_amdgcn_readfirstlane(ld32(&ov_slot[j]));
            }
            ReqHdr* nh = ov_hdr + (size_t)s * K;
            uint64_t* nwd = ov_words + (size_t)s * d.DW;
            if (from_ws) {
                if (lane < S.CC.nck) {
                    const int kk = S.CC.key[lane];
                    nh[kk] = S.ws.hdr[lane];
                    for (int i = 0; i < S.CC.nw[lane]; i++) nwd[S.CC.woff[lane] + i] = S.ws.words[S.CC.wsoff[lane] + i];
                }
            } else {
                for (int i = d.cls_xkoff[c] + lane; i < d.cls_xkoff[c + 1]; i += 64) {
                    const int kk = d.cls_xkeys[i];
                    ReqHdr a = nh[kk];
                    req_merge_inplace(d, kk, a, nwd + d.woff[kk], d.cls_hdr[(size_t)c * K + kk],
                                      d.cls_words + (size_t)c * d.DW + d.woff[kk]);
                    nh[kk] = a;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        };
        auto scan_nodes = [&](int c, const int64_t (&q)[KP_LDS_AXES], int xs, bool tcons, const int64_t* pr) -> int {
            int jf = -1;
            uint64_t fmask = 0;
            int fgrp = -1;
            for (int base = __builtin_amdgcn_readfirstlane(xs & ~63); base < E; base += 64) {
                const int w = base >> 6;
                const int j = base + lane;
                if (base != cbase && k.use_cmax) {
                    if ((w >> 6) != fgrp) {
                        fgrp = w >> 6;
                        const int wl = (fgrp << 6) + lane;
                        bool pc = false;
                        if (wl < EW) {
                            const uint64_t mx = (MUT && mutp) ? mutn[wl] : 0ull;  // changed nodes: maybe compatible
                            pc = ((d.XT[(size_t)c * EW + wl] | mx) & ~excl[wl]) != 0;
#pragma unroll
                            for (int ai = 0; ai < KP_LDS_AXES; ai++)
                                if (ai < A) pc = pc && q[ai] <= cmax[wl * KP_LDS_AXES + ai];
                        }
                        fmask = ballot(pc);
                    }
                    if (!((fmask >> (w & 63)) & 1ull)) {  // no node of the chunk can take the pod
                        const uint64_t rest = fmask & ~((2ull << (w & 63)) - 1ull);
                        const int nxt = rest ? (fgrp << 6) + __ffsll((unsigned long long)rest) - 1 : (fgrp + 1) << 6;
                        st_skips += nxt - w;
                        base = __builtin_amdgcn_readfirstlane((nxt << 6) - 64);
                        continue;
                    }
                }
                const uint64_t ge = xs > base ? (~0ull << (xs - base)) : ~0ull;
                uint64_t xw, mw = 0;
                int64_t h[KP_LDS_AXES], dl[KP_LDS_AXES];
                bool fresh = false;
                if (base == cbase) {
                    st_hits++;
                    if (ccls != c) {
                        cx = uni64((d.C <= KP_CONS_XTC) ? xtc[c] : (d.XT[(size_t)c * EW + w] & ~excl[w]));
                        ccls = c;
                    }
                    xw = mut_patch(c, w, cx);
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                        h[ai] = ch[ai];
                        dl[ai] = cd[ai];
                    }
                } else {
                    xw = mut_patch(c, w, uni64(d.XT[(size_t)c * EW + w] & ~excl[w]));
                    if (!(xw & ge)) {
                        st_nodes += 64;
                        continue;
                    }
                    st_loads++;
                    fresh = true;
                    mw = uni64(modb[w]);  // not the cached chunk's word: LDS is current
                    // the static headroom first: its loads are in flight while the delta stores drain
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                        h[ai] = 0;
                        dl[ai] = 0;
                        if (ai < A && j < E) h[ai] = d.ex_head[(size_t)ai * E + j];
                    }
                    if (mw) {
                        if (mw & xw) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this probe's delta stores landed
                        const bool md = (mw >> lane) & 1ull;
#pragma unroll
                        for (int ai = 0; ai < KP_LDS_AXES; ai++)
                            if (ai < A && j < E && md) dl[ai] = ld_req(&delta[(size_t)ai * E + j]);
                    }
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) h[ai] -= dl[ai];
                }
                bool cand = (xw & ge) >> lane & 1ull;
#pragma unroll
                for (int ai = 0; ai < KP_LDS_AXES; ai++)
                    if (ai < A) cand &= q[ai] <= h[ai];
                if (wide && ballot(cand)) {
                    const bool md = (((base == cbase) ? cmod : mw) >> lane) & 1ull;
                    for (int ai = KP_LDS_AXES; ai < A && cand; ai++) {
                        int64_t hx = d.ex_head[(size_t)ai * E + j];
                        if (md) hx -= ld_req(&delta[(size_t)ai * E + j]);
                        cand = pr[d.active_axes[ai]] <= hx;
                    }
                }
                st_nodes += 64;
                uint64_t m = ballot(cand);
                if (TOPO && tcons) {  // ExistingNode.Add's topology step on each fitting node, in order
                    while (m) {
                        const int jj = __builtin_amdgcn_readfirstlane(base + __ffsll((unsigned long long)m) - 1);
                        const ReqHdr* nh;
                        const uint64_t* nwd;
                        node_digest(jj, nh, nwd);
                        if (existing_topo_try<true, true>(d, S.CC, S.ws, jj, lane, &P, nh, nwd)) break;
                        m &= m - 1;
                    }
                    m = uni64(m);
                }
                if (m) {
                    jf = __builtin_amdgcn_readfirstlane(base + __ffsll((unsigned long long)m) - 1);
                    if (base != cbase) {
                        // evict: this probe's requests on the old chunk go to the delta slab (read back past L1), its
                        // headroom maximum to the summary
                        if (cbase >= 0) {
                            if (lane == 0) modb[cbase >> 6] = cmod;
                            if (k.use_cmax)
#pragma unroll
                                for (int ai = 0; ai < KP_LDS_AXES; ai++)
                                    if (ai < A) {
                                        const int64_t mx = chunk_max(cbase, ch, ai);
                                        if (lane == 0) cmax[(cbase >> 6) * KP_LDS_AXES + ai] = mx;
                                    }
                        }
                        if (cbase >= 0 && ((cmod >> lane) & 1ull)) {
#pragma unroll
                            for (int ai = 0; ai < KP_LDS_AXES; ai++)
                                if (ai < A)
                                    __hip_atomic_store(&delta[(size_t)ai * E + cbase + lane], cd[ai], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                        }
                        if (d.C <= KP_CONS_XTC)
                            for (int cc = lane; cc < d.C; cc += 64) xtc[cc] = d.XT[(size_t)cc * EW + w] & ~excl[w];
                        cbase = base;
                        cx = xw;
                        ccls = c;
                        cmod = mw;
                        cinit = uni64(initb[w]);
#pragma unroll
                        for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                            ch[ai] = h[ai];
                            cd[ai] = dl[ai];
                        }
                    }
                    break;
                }
                if (fresh && k.use_cmax)  // the loaded chunk cannot take the pod: its summary entry drops to its maximum
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++)
                        if (ai < A) {
                            const int64_t mx = chunk_max(base, h, ai);
                            if (lane == 0) cmax[w * KP_LDS_AXES + ai] = mx;
                        }
            }
            return jf;
        };
        if (!TOPO && !serial) {
            // ---- existing nodes: the probe's pods in windows of 64, one pod per lane ----
            // Fast variant: every pod here lands on an existing node or the probe goes to the FULL variant, so the queue
            // is one pass in order and the probe is plain first fit: each pod takes the first node in scheduling order
            // that is compatible, not a candidate, and has headroom for it.  FULL variant: the same pass runs first and
            // records which pods no existing node takes (k.pnode); ExistingNode.Add is independent of the in-flight
            // NodeClaim, existing nodes only lose headroom, and a pod is first popped in queue order, so these are the
            // placements the serial queue below would make, and a pod refused once (or re-pushed later) is refused by
            // every node again: the queue then runs NodeClaim.Add / the templates for those pods only.  First fit is computed node-major: node j, in order,
            // takes from the window's pods not yet placed, in queue order, each one that still fits it (a pod that first
            // fits node j under pod-major first fit is exactly one node j takes here: by induction over j, the pods an
            // earlier node took before pod i are the same in both orders).  Per node the intake is greedy in queue
            // order over the pods that fit it on their own: when there are many, one round of inclusive prefix sums
            // takes the prefix up to the first running-total overflow, and a scalar pass over the few later pods that
            // still fit what is left finishes it.  The first KS chunks live in an LDS store for the probe (hs: headroom
            // per axis and node, loaded on first touch, updated in place); a pod that fits no store node takes the serial
            // scan over the later chunks, in queue order.
            const int KS = k.n_store;
            const int AA = NA > 0 ? NA : A;  // active axes (compile-time in the NA instantiations)
            const int SE = KS * 64 < E ? KS * 64 : E;  // nodes [0, SE) are in the store
            int64_t* hs = reinterpret_cast<int64_t*>(smem + k.off_hs);  // [KS][A][64]
            uint64_t loaded = 0;  // store chunks in LDS
            const long long cf0 = prof ? __builtin_amdgcn_s_memtime() : 0;
            int32_t* pnode = FULL ? k.pnode + (size_t)wid * cap : nullptr;
            for (int wb = 0; wb < n && !aborted; wb += 64) {
                const long long cw0 = prof ? __builtin_amdgcn_s_memtime() : 0;
                const int wn = __builtin_amdgcn_readfirstlane(n - wb < 64 ? n - wb : 64);
                const bool live = lane < wn;
                const int went = live ? ld32(&ring[wb + lane]) : 0;
                const int wp = went & 0x7fffffff;
                const bool wpend = went < 0;
                const int wc = live ? pcls[wp] : 0;
                int64_t wq[KP_LDS_AXES];
#pragma unroll
                for (int ai = 0; ai < KP_LDS_AXES; ai++)
                    wq[ai] = (live && ai < A) ? d.pod_req[(size_t)wp * R + d.active_axes[ai]] : 0;
                st_pops += wn;
                const uint64_t pendm = ballot(live && wpend);
                if (prof) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    pf_load += __builtin_amdgcn_s_memtime() - cw0;
                }
                uint64_t U = ballot(live);  // pods of the window not placed yet
                // this pod's compatible-node words, one chunk ahead (the next chunk's load is in flight while this one is
                // taken)
                uint64_t xnext = (live && KS > 0) ? d.XT[(size_t)wc * EW] : 0ull;
                // smallest request per axis over the window's pods not placed yet (recomputed when U changes)
                int64_t mq[KP_LDS_AXES];
                uint64_t mqU = 0;
#pragma unroll
                for (int ai = 0; ai < KP_LDS_AXES; ai++) mq[ai] = 0;
                for (int w = 0; w < KS && U; w++) {
                    const long long cc0 = prof ? __builtin_amdgcn_s_memtime() : 0;
                    const bool inU = (U >> lane) & 1ull;
                    const uint64_t xw = inU ? (xnext & ~excl[w]) : 0ull;  // this pod's nodes
                    xnext = (live && w + 1 < KS) ? d.XT[(size_t)wc * EW + w + 1] : 0ull;
                    const uint64_t anyc = uni64(wave_or64(xw));
                    if (!anyc) continue;
                    if (!((loaded >> w) & 1ull)) {  // first touch: the chunk's headroom into the store
                        const int j = w * 64 + lane;
                        AXL(ai) hs[(w * AA + ai) * 64 + lane] = j < E ? d.ex_head[(size_t)ai * E + j] : -1;
                        loaded |= 1ull << w;
                        st_loads++;
                    }
                    // a node below the smallest remaining request on some axis takes none of them
                    if (U != mqU) {
                        mqU = U;
                        AXL(ai) mq[ai] = (int64_t)wave_reduce64(inU ? (uint64_t)wq[ai] : (uint64_t)INT64_MAX,
                                                                [](uint64_t a, uint64_t b) { return (int64_t)b < (int64_t)a ? b : a; });
                    }
                    bool pot = (anyc >> lane) & 1ull;
                    int64_t hl[KP_LDS_AXES];
                    AXL(ai) {
                            hl[ai] = hs[(w * AA + ai) * 64 + lane];
                            pot = pot && hl[ai] >= mq[ai];
                        }
                    st_nodes += 64;
                    const uint64_t iw = uni64(initb[w]);
                    uint64_t touched = 0;
                    const long long cn0 = prof ? __builtin_amdgcn_s_memtime() : 0;
                    if (prof) pf_prep += cn0 - cc0;
                    for (uint64_t m = ballot(pot); m && U; m &= m - 1) {
                        const int jn = __ffsll((unsigned long long)m) - 1;
                        pf_visits++;
                        int64_t hj[KP_LDS_AXES];
#pragma unroll
                        for (int ai = 0; ai < KP_LDS_AXES; ai++) hj[ai] = ai < A ? (int64_t)rl64((uint64_t)hl[ai], jn) : 0;
                        // the pods that fit the node on their own; a pod outside this set never fits it later
                        bool e = ((U >> lane) & 1ull) && ((xw >> jn) & 1ull);
                        AXL(ai) e = e && wq[ai] <= hj[ai];
                        uint64_t em = ballot(e);
                        if (!em) continue;
                        uint64_t took = 0;
                        if (__popcll(em) > 4) {
                            pf_many++;
                            // many: the prefix up to the first running-total overflow is taken in one round of prefix sums
                            bool over = false;
                            int64_t pv[KP_LDS_AXES];
                            AXL(ai) {
                                    pv[ai] = (int64_t)wave_scan_add64(e ? (uint64_t)wq[ai] : 0ull);
                                    over = over || pv[ai] > hj[ai];
                                }
                            const uint64_t ov = ballot(e && over);
                            const int fo = ov ? __ffsll((unsigned long long)ov) - 1 : 64;
                            took = em & (fo >= 64 ? ~0ull : ((1ull << fo) - 1ull));
                            if (took) {
                                const int last = 63 - __clzll((long long)took);
                                AXL(ai) hj[ai] -= (int64_t)rl64((uint64_t)pv[ai], last);
                            }
                            // the rest: the pods after the overflowing one that still fit what is left
                            bool e2 = e && lane > fo;
                            AXL(ai) e2 = e2 && wq[ai] <= hj[ai];
                            em = fo >= 64 ? 0ull : ballot(e2);
                        }
                        // few: greedily in queue order with scalar running totals
                        for (; em; em &= em - 1) {
                            const int t = __ffsll((unsigned long long)em) - 1;
                            pf_iters++;
                            int64_t qt[KP_LDS_AXES];
                            bool ok = true;
                            AXL(ai) {
                                    qt[ai] = (int64_t)rl64((uint64_t)wq[ai], t);
                                    ok = ok && qt[ai] <= hj[ai];
                                }
                            if (!ok) continue;
                            AXL(ai) hj[ai] -= qt[ai];
                            took |= 1ull << t;
                        }
                        if (!took) continue;
                        U &= ~took;
                        touched |= 1ull << jn;
                        AXL(ai) if (lane == jn) hl[ai] = hj[ai];
                        const int ntk = __popcll(took);
                        st_placed += ntk;
                        st_hits += ntk;
                        // SimulateScheduling: a non-pending pod placed on an uninitialized node is an error
                        const uint64_t npl = took & ~pendm;
                        if ((iw >> jn) & 1ull) ok_np += __popcll(npl);
                        else if (npl) bad = true;
                    }
                    if ((touched >> lane) & 1ull) {  // each lane writes back its own node
                        AXL(ai) hs[(w * AA + ai) * 64 + lane] = hl[ai];
                    }
                    if (prof) pf_nodes += __builtin_amdgcn_s_memtime() - cn0;
                }
                // the pods no store node takes: the chunks after the store, serially in queue order
                const long long cm0 = prof ? __builtin_amdgcn_s_memtime() : 0;
                if (prof) pf_miss += __popcll(U);
                for (uint64_t m = U; m && !aborted; m &= m - 1) {
                    const int i = __ffsll((unsigned long long)m) - 1;
                    const int c = rl32(wc, i);
                    const int shape = pshape[rl32(wp, i)];
                    const bool pend = (pendm >> i) & 1ull;
                    int64_t q[KP_LDS_AXES];
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) q[ai] = (int64_t)rl64((uint64_t)wq[ai], i);
                    if (shape != prev_shape) {
                        prev_shape = shape;
                        xstart = 0;
                    }
                    const int jf = SE < E ? scan_nodes(c, q, xstart > SE ? xstart : SE, false, nullptr) : -1;
                    if (jf < 0) {
                        if constexpr (!FULL) {
                            aborted = true;  // needs a NodeClaim: the FULL variant redoes this probe
                            break;
                        } else {
                            xstart = E;  // every node refuses this shape from now on
                            continue;
                        }
                    }
                    U &= ~(1ull << i);
                    if (lane == jf - cbase) {
                        AXL(ai) {
                                ch[ai] -= q[ai];
                                cd[ai] += q[ai];
                            }
                    }
                    cmod |= 1ull << (jf & 63);
                    xstart = jf;
                    st_placed++;
                    if (!pend) {
                        if ((cinit >> (jf & 63)) & 1ull) ok_np++;
                        else bad = true;
                    }
                }
                if (prof) pf_miss_cyc += __builtin_amdgcn_s_memtime() - cm0;
                if (FULL && live) pnode[wb + lane] = ((U >> lane) & 1ull) ? -1 : 0;
            }
            if (FULL && k.relax) {
                // a relaxed pod is offered to the existing nodes again by scan_nodes, which reads headroom as ex_head
                // minus this probe's delta slab: the store chunks' headroom goes there
                for (int w = 0; w < KS; w++) {
                    if (!((loaded >> w) & 1ull)) continue;
                    const int j = w * 64 + lane;
                    if (j < E)
                        AXL(ai) __hip_atomic_store(&delta[(size_t)ai * E + j], d.ex_head[(size_t)ai * E + j] - hs[(w * AA + ai) * 64 + lane],
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (lane == 0) modb[w] = ~0ull;
                }
                __syncthreads();
            }
            if (FULL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (prof) cy_scan = __builtin_amdgcn_s_memtime() - cf0;
        }
        if constexpr (FULL || TOPO) while (count > 0 && !aborted) {
            // loop-carried wave-uniform state: re-asserted scalar each pod, so the chunk tests below branch on SGPRs
            head = __builtin_amdgcn_readfirstlane(head);
            count = __builtin_amdgcn_readfirstlane(count);
            wbase = __builtin_amdgcn_readfirstlane(wbase);
            xstart = __builtin_amdgcn_readfirstlane(xstart);
            cbase = __builtin_amdgcn_readfirstlane(cbase);
            ccls = __builtin_amdgcn_readfirstlane(ccls);
            prev_shape = __builtin_amdgcn_readfirstlane(prev_shape);
            cx = uni64(cx);
            cmod = uni64(cmod);
            cinit = uni64(cinit);
            relax_at = __builtin_amdgcn_readfirstlane(relax_at);
            if (head - wbase >= 64) win_load(head);
            const int off = head - wbase;
            const int pos0 = head;
            const int ent = rl32(vpod, off);
            const int elast = pos0 <= relax_at ? -1 : rl32(vlast, off);
            if (elast == count) break;  // Queue.Pop: cycled through the queue without progress
            head++;
            count--;
            // FULL, no topology: the window pass above placed this pod on an existing node (first pop), or every node
            // refuses it
            if (FULL && !TOPO && !serial && pos0 < n && rl32(vpn, off) >= 0) continue;
            st_pops++;
            const bool pend = ent < 0;
            const int p = ent & 0x3fffffff;
            const int cf = rl32(vc, off);
            const int c = cf & 0x7fffffff;
            const bool fresh = cf < 0;  // a relaxed class the existing nodes have not been offered yet
            const int shape = rl32(vshape, off);
            int64_t q[KP_LDS_AXES];
#pragma unroll
            for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                const uint32_t lo = (uint32_t)rl32((int)(uint32_t)vq[ai], off);
                const uint32_t hi = (uint32_t)rl32((int)(uint32_t)((uint64_t)vq[ai] >> 32), off);
                q[ai] = (int64_t)(((uint64_t)hi << 32) | lo);
            }
            if (shape != prev_shape) {  // nodes before xstart rejected this shape and only lose headroom
                prev_shape = shape;
                xstart = 0;
            }
            // TOPO: a class counted by some group records each placement; a constrained class's node rejections depend
            // on counts (scan from the first node, no resume)
            uint32_t cflags = 0;
            if (TOPO) {
                cflags = __builtin_amdgcn_readfirstlane(d.cls_flags[c]);
                if ((cflags & CF_TOPO) && S.CC.cls != c) fill_class_cache<TOPO>(d, c, S.CC, lane, 64, TOPO ? S.born : 0ull);
            }
            const bool tcons = TOPO && (cflags & CF_TOPO_CONS);
            const int xs = tcons ? 0 : xstart;
            const long long cs0 = prof ? __builtin_amdgcn_s_memtime() : 0;
            const int jf = (FULL && !TOPO && !fresh && !serial) ? -1 : scan_nodes(c, q, xs, tcons, d.pod_req + (size_t)p * R);
            if (prof) cy_scan += __builtin_amdgcn_s_memtime() - cs0;
            if (jf >= 0) {
                if (wide && lane == 0) {  // the axes past the registers: this probe's delta slab, valid from the first pod
                    const bool was = (cmod >> (jf & 63)) & 1ull;
                    for (int ai = KP_LDS_AXES; ai < A; ai++) {
                        int64_t* dp = &delta[(size_t)ai * E + jf];
                        __hip_atomic_store(dp, (was ? ld_req(dp) : 0) + d.pod_req[(size_t)p * R + d.active_axes[ai]],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                if (lane == jf - cbase) {
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                        if (ai < A) {
                            ch[ai] -= q[ai];
                            cd[ai] += q[ai];
                        }
                    }
                }
                cmod |= 1ull << (jf & 63);  // jf lies in the cached chunk
                if (!tcons) xstart = jf;
                if (TOPO && (cflags & CF_TOPO)) {  // Topology.Record with the node's merged requirements and taints
                    const ReqHdr* nh;
                    const uint64_t* nwd;
                    node_digest(jf, nh, nwd);
                    if (!tcons) existing_topo_try<false, true>(d, S.CC, S.ws, jf, lane, &P, nh, nwd);
                    topo_record<true>(d, S.CC, S.ws, nh, nwd, jf, -1, false, lane, jf, &P);
                }
                if (MUT && mutp) mut_commit(c, jf, TOPO && (cflags & CF_TOPO));
                st_placed++;
                if (!pend) {
                    if ((cinit >> (jf & 63)) & 1ull) ok_np++;
                    else bad = true;  // SimulateScheduling: uninitialized-node placement is an error
                }
                continue;
            }
            if (!tcons) xstart = E;
            if constexpr (!FULL) {
                aborted = true;  // needs a NodeClaim: the FULL variant redoes this probe
                break;
            }
            bool placed = false;
            const long long cn0 = prof ? __builtin_amdgcn_s_memtime() : 0;
            const int64_t* preq = d.pod_req + (size_t)p * R;
            if (n_nc == 1) {  // NodeClaim.Add on the in-flight NodeClaim
                if (S.CC.cls != c) fill_class_cache<TOPO>(d, c, S.CC, lane, 64, TOPO ? S.born : 0ull);
                EvalIn a;
                a.Ahdr = nch;
                a.Aw = ncw;
                a.opts = nc_opts;
                a.base_req = S.nc_req;
                a.pod_req = preq;
                a.tmpl = nc_tmpl;
                a.compat = true;
                a.force_off = false;
                a.prof = nullptr;
                a.host = E;  // the in-flight NodeClaim's hostname row
                a.held = nc_held;
                st_nc++;
                // the NodeClaim has absorbed the class (no topology, no reservations): the merge is idempotent and the
                // label / offering filters already hold for its options, so the Add is Fits (+ minValues) only
                bool absorbed = c == nc_lc && !(TOPO && (cflags & CF_TOPO)) && !(RESV && d.resv_on);
                // another class whose requirement merge changes nothing (and that tolerates the NodeClaim's template)
                // is absorbed the same way
                if (!absorbed && !(TOPO && (cflags & CF_TOPO)) && !(RESV && d.resv_on) && ((d.tol[c] >> nc_tmpl) & 1ull) &&
                    merge_noop_at(d, S.ws, nch, ncw, c, lane)) {
                    absorbed = true;
                    nc_lc = c;  // its requirements are a subset of the class's
                }
                if (absorbed) {
                    if (eval_fits_only<true>(d, Ev, a, S.ws, lane)) {
                        if (lane < TW) nc_opts = S.ws.opts[lane];
                        if (lane < R) S.nc_req[lane] += preq[lane];
                        __syncthreads();
                        if (d.best_effort) commit_min_relax_lds(nch, S.ws, lane);
                        placed = true;
                    }
                } else if (tcons ? eval_wave<true, RESV, false, true, true>(d, Ev, S.CC, a, S.ws, lane)
                                 : eval_wave<false, RESV, false>(d, Ev, S.CC, a, S.ws, lane)) {
                    nc_lc = c;
                    if (lane < S.CC.nck) {
                        const int kk = S.CC.key[lane];
                        nch[kk] = S.ws.hdr[lane];
                        for (int i = 0; i < S.CC.nw[lane]; i++) ncw[S.CC.woff[lane] + i] = S.ws.words[S.CC.wsoff[lane] + i];
                    }
                    if (lane < TW) nc_opts = S.ws.opts[lane];
                    if (lane < R) S.nc_req[lane] += preq[lane];
                    if (RESV && d.resv_on) nc_held = commit_held(rcap, nc_held, S.ws, d.ro_ridw, lane);
                    __syncthreads();
                    if (d.best_effort) commit_min_relax_lds(nch, S.ws, lane);
                    if (TOPO && (cflags & CF_TOPO)) topo_record<true>(d, S.CC, S.ws, nch, ncw, E, nc_tmpl, true, lane, -1, &P);
                    placed = true;
                }
            }
            if (!placed) {  // new NodeClaim from the templates in weight order
                for (int j = 0; j < NT; j++) {
                    uint64_t o = (lane < TW && d.tmpl_ok[j]) ? d.tmpl_opts[(size_t)j * TW + lane] : 0;
                    o = limit_filter_rem(d, j, o, rem, lane);
                    if (!ballot(o != 0)) continue;
                    if (S.CC.cls != c) fill_class_cache<TOPO>(d, c, S.CC, lane, 64, TOPO ? S.born : 0ull);
                    EvalIn a;
                    a.Ahdr = d.cls_hdr + (size_t)(d.C + j) * K;
                    a.Aw = d.cls_words + (size_t)(d.C + j) * d.DW;
                    a.opts = o;
                    a.base_req = d.daemon + (size_t)j * R;
                    a.pod_req = preq;
                    a.tmpl = j;
                    a.compat = true;
                    a.force_off = false;
                    a.prof = nullptr;
                    a.host = E + 1;  // a new NodeClaim's hostname: no pod counted there yet
                    a.held = 0;
                    st_tmpl++;
                    if (!(tcons ? eval_wave<true, RESV, false, true, true>(d, Ev, S.CC, a, S.ws, lane)
                                : eval_wave<false, RESV, false>(d, Ev, S.CC, a, S.ws, lane)))
                        continue;
                    if (n_nc == 1) {  // a second NodeClaim: computeConsolidation returns NONE
                        stop = true;
                        break;
                    }
                    for (int kk = lane; kk < K; kk += 64) nch[kk] = d.cls_hdr[(size_t)(d.C + j) * K + kk];
                    for (int i = lane; i < d.DW; i += 64) ncw[i] = d.cls_words[(size_t)(d.C + j) * d.DW + i];
                    __syncthreads();
                    if (lane < S.CC.nck) {
                        const int kk = S.CC.key[lane];
                        nch[kk] = S.ws.hdr[lane];
                        for (int i = 0; i < S.CC.nw[lane]; i++) ncw[S.CC.woff[lane] + i] = S.ws.words[S.CC.wsoff[lane] + i];
                    }
                    nc_opts = lane < TW ? S.ws.opts[lane] : 0;
                    if (lane < R) S.nc_req[lane] = d.daemon[(size_t)j * R + lane] + preq[lane];
                    if (RESV && d.resv_on) nc_held = commit_held(rcap, 0ull, S.ws, d.ro_ridw, lane);
                    // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
                    for (int r = 0; r < R; r++) {
                        if (!d.limit_set[(size_t)j * R + r]) continue;
                        int64_t mx = INT64_MIN;
                        for (int w = 0; w < TW; w++) {
                            const uint64_t ow = rl64(nc_opts, w);
                            if ((ow >> lane) & 1ull) {
                                const int64_t cp = d.cap[(size_t)r * T + w * 64 + lane];
                                mx = cp > mx ? cp : mx;
                            }
                        }
                        mx = wave_max64(mx);
                        if (lane == 0) rem[j * R + r] -= mx;
                    }
                    nc_tmpl = j;
                    n_nc = 1;
                    nc_lc = c;
                    placed = true;
                    __syncthreads();
                    if (d.best_effort) commit_min_relax_lds(nch, S.ws, lane);
                    if (TOPO) {  // the NodeClaim's hostname row starts empty; Record the pod
                        for (int r = lane; r < k.HG; r += 64)
                            __hip_atomic_store(&P.hd[(size_t)r * (E + 1) + E], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (cflags & CF_TOPO) topo_record<true>(d, S.CC, S.ws, nch, ncw, E, j, true, lane, -1, &P);
                    }
                    break;
                }
            }
            if (prof) cy_nc += __builtin_amdgcn_s_memtime() - cn0;
            if (stop) break;
            if (placed) {
                if (!pend) {
                    ok_np++;
                    nc_nonpend++;
                }
                continue;
            }
            // preferences.Relax, then Queue.Push(pod, relaxed): a relaxed pod takes its class's next stage (fresh: the
            // existing nodes see it again) and clears every lastLen; otherwise lastLen = len after the append
            const int tail = head + count;
            const int nx = k.relax ? d.relax_next[c] : -1;
            const int nent = k.relax ? (ent | 0x40000000) : ent;
            const int ncls = nx >= 0 ? (nx | (int)0x80000000) : c;
            const int nshape = nx >= 0 ? d.shape_next[shape] : shape;
            const int nlast = nx >= 0 ? -1 : count + 1;
            if (nx >= 0) {
                relax_at = tail;
                st_relax++;
                // Topology.Update: the relaxed spec's new groups are created (one wave: its LDS ops stay in order)
                if (TOPO && d.tg_late && lane == 0) S.born = topo_birth(d, S.born, d.cls_birth[nx]);
            }
            if (lane == 0) {
                ring[tail % cap] = nent;
                rlast[tail % cap] = nlast;
                if (k.relax) {
                    rcls[tail % cap] = ncls;
                    rshape[tail % cap] = nshape;
                }
            }
            if (tail - wbase < 64 && lane == tail - wbase) {
                vpod = nent;
                vlast = nlast;
                vc = ncls;
                vshape = nshape;
#pragma unroll
                for (int ai = 0; ai < KP_LDS_AXES; ai++) vq[ai] = q[ai];
            }
            count++;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }

        if (!FULL && aborted) {
            if (lane == 0) {
                const int slot = atomicAdd(&k.next_probe[2], 1);
                k.retry[slot] = probe;
            }
        } else {
        // ---- computeConsolidation ----
        const long long cd0 = prof ? __builtin_amdgcn_s_memtime() : 0;
        int decision = KP_DECISION_NONE, valid = 0, nrep = 0;
        double rprice = 0.0;
        bool truncated_out = false;  // the NodeClaim failed TruncateInstanceTypes' minValues check
        const bool all = !stop && !bad && ok_np == n_np;
        if (all && n_nc == 0) {
            decision = KP_DECISION_DELETE;
            valid = 1;
        } else if (FULL && all) {
            // FinalizeScheduling: a NodeClaim holding reservations gets reservation-id In [held IDs]
            if (RESV && ballot(nc_held != 0) && d.key_resvid >= 0) {
                if (lane == 0) {
                    ReqHdr h{};
                    h.flags = RF_DEF;
                    nch[d.key_resvid] = h;
                }
                for (int i = lane; i < d.nw[d.key_resvid]; i += 64) ncw[d.woff[d.key_resvid] + i] = 0ull;
                __syncthreads();
                for (uint64_t x = lane < d.ro_ridw ? nc_held : 0ull; x; x &= x - 1) {  // the held IDs' value bits
                    const int v = d.ro->rid_vid[lane * 64 + __ffsll((unsigned long long)x) - 1];
                    atomicOr((unsigned long long*)&ncw[d.woff[d.key_resvid] + (v >> 6)], 1ull << (v & 63));
                }
                __syncthreads();
            }
            // Offerings.Available().Compatible(NodeClaim requirements) over zone × capacity-type slots
            bool okslot = false;
            if (lane < d.n_slots) {
                auto adm = [&](int kk, int v) -> bool {
                    if (kk < 0) return true;
                    const ReqHdr h = nch[kk];
                    if (!(h.flags & RF_DEF)) return true;
                    return req_has(d, kk, v, h, ncw + d.woff[kk]);
                };
                auto dneok = [&](int kk) -> bool {
                    if (kk < 0) return true;
                    const ReqHdr h = nch[kk];
                    if (!(h.flags & RF_DEF)) return true;
                    return op_notin_or_dne(req_op(h.flags, popc_words(ncw + d.woff[kk], d.nw[kk])));
                };
                okslot = adm(d.key_zone, d.slot_zone[lane]) && adm(d.key_ct, d.slot_ct[lane]) &&
                         (d.slot_zoneid[lane] < 0 || adm(d.key_zoneid, d.slot_zoneid[lane])) && dneok(d.key_resvid) &&
                         dneok(d.key_resvtype);
            }
            const uint64_t mzc = ballot(okslot);
            // ... and over the reserved offerings (capacity-type In [reserved], zone, zone-id, reservation id / type), 64
            // rows per step into S.mro
            for (int q = 0; RESV && q < d.ro_w; q++) {
                const int ri = q * 64 + lane;
                bool ok = false;
                if (ri < d.ro_n && d.ro->type[ri] >= 0 && ((d.ro->avail[q] >> lane) & 1ull)) {
                    auto adm = [&](int kk, int v) -> bool {
                        if (kk < 0) return true;
                        const ReqHdr h = nch[kk];
                        if (!(h.flags & RF_DEF)) return true;
                        return req_has(d, kk, v, h, ncw + d.woff[kk]);
                    };
                    const int zid = d.ro->zid[ri], rt = d.ro->rtype[ri];
                    bool rtok;
                    if (rt >= 0) {
                        rtok = adm(d.key_resvtype, rt);
                    } else {
                        const int kk = d.key_resvtype;
                        const ReqHdr h = kk >= 0 ? nch[kk] : ReqHdr{};
                        rtok = kk < 0 || !(h.flags & RF_DEF) ||
                               op_notin_or_dne(req_op(h.flags, popc_words(ncw + d.woff[kk], d.nw[kk])));
                    }
                    ok = adm(d.key_ct, d.ro->ctv) && adm(d.key_zone, d.ro->zone[ri]) && (zid < 0 || adm(d.key_zoneid, zid)) &&
                         adm(d.key_resvid, d.ro->ridv[ri]) && rtok;
                }
                const uint64_t m = ballot(ok);
                if (lane == 0) S.mro[q] = m;
            }
            if (RESV) __syncthreads();
            // OrderByPrice(reqs) + Truncate(M): select the M cheapest options by (price, name)
            double pr[KP_TW_MAX];
            uint32_t rk[KP_TW_MAX];
            uint32_t present = 0;
            int n_opt = 0;
#pragma unroll
            for (int w = 0; w < KP_TW_MAX; w++) {
                pr[w] = DBL_MAX;
                rk[w] = 0xFFFFFFFFu;
                if (w < TW) {
                    const uint64_t word = rl64(nc_opts, w);
                    n_opt += __popcll(word);
                    if ((word >> lane) & 1ull) {
                        const int t = w * 64 + lane;
                        uint64_t m = d.avail_zc[t] & mzc;
                        double price = DBL_MAX;
                        while (m) {
                            const int s = __ffsll((unsigned long long)m) - 1;
                            m &= m - 1;
                            const double sp = d.slot_price[(size_t)t * KP_MAX_SLOTS + s];
                            price = sp < price ? sp : price;
                        }
                        if (RESV) {
                            const uint32_t tr = d.type_ro[t];
                            for (uint64_t x = tr ? S.mro[tr >> 16] & ro_span_bits(tr) : 0ull; x; x &= x - 1) {
                                const double rp = d.ro_price[(tr >> 16) * 64 + __ffsll((unsigned long long)x) - 1];
                                price = rp < price ? rp : price;
                            }
                        }
                        pr[w] = price;
                        rk[w] = d.name_rank[t];
                        present |= 1u << w;
                    }
                }
            }
            const int nsel = n_opt < d.M ? n_opt : d.M;
            const bool has_min = (Ev.min_tmpl_mask >> nc_tmpl) & 1ull;
            int my_t = -1;
            for (int i = 0; i < nsel; i++) {
                double bp = DBL_MAX;
                uint32_t br = 0xFFFFFFFFu;
                int bw = -1;
#pragma unroll
                for (int w = 0; w < KP_TW_MAX; w++) {
                    if (((present >> w) & 1u) && (bw < 0 || pr[w] < bp || (pr[w] == bp && rk[w] < br))) {
                        bp = pr[w];
                        br = rk[w];
                        bw = w;
                    }
                }
                int gl = bw >= 0 ? lane : -1, gw = bw;
                for (int o = 32; o >= 1; o >>= 1) {
                    const double op = __shfl_xor(bp, o);
                    const uint32_t orr = (uint32_t)__shfl_xor((int)br, o);
                    const int ol = __shfl_xor(gl, o), ow = __shfl_xor(gw, o);
                    if (ol >= 0 && (gl < 0 || op < bp || (op == bp && orr < br))) {
                        bp = op;
                        br = orr;
                        gl = ol;
                        gw = ow;
                    }
                }
                gl = __builtin_amdgcn_readfirstlane(gl);
                gw = __builtin_amdgcn_readfirstlane(gw);
                if (lane == i) my_t = gw * 64 + gl;
                if (lane == gl) present &= ~(1u << gw);
            }
            // Results.TruncateInstanceTypes: a NodeClaim whose first M options miss its minValues is dropped and its pods
            // get errors (not every non-pending pod scheduled; no valid new NodeClaim)
            const uint64_t msel = nsel >= 64 ? ~0ull : ((1ull << nsel) - 1);
            const bool trunc_ok = !has_min || min_values_ok(d, nch, nc_tmpl, my_t, msel, lane, nullptr);
            // capacity-type requirement of the NodeClaim: Has(spot) / Has(on-demand)
            auto ct_has = [&](int vid) -> bool {
                const int kk = d.key_ct;
                if (kk < 0) return true;
                const ReqHdr h = nch[kk];
                if (!(h.flags & RF_DEF)) return true;  // undefined: Get() is Exists
                if (vid < 0) return (h.flags & RF_CMP) && !(h.flags & (RF_GT | RF_LT));
                return req_has(d, kk, vid, h, ncw + d.woff[kk]);
            };
            const bool has_spot = ct_has(k.v_spot), has_od = ct_has(k.v_od);
            const uint64_t mt = my_t >= 0 ? d.avail_zc[my_t] & mzc : 0;
            // the option's reserved offerings (bits of ResvTab word mrw)
            const uint32_t mtr = (RESV && my_t >= 0) ? d.type_ro[my_t] : 0u;
            const uint64_t mr = mtr ? S.mro[mtr >> 16] & ro_span_bits(mtr) : 0ull;
            const int mrw = (int)(mtr >> 16);
            bool keep = false, none = false, spot_only = false;
            if (!trunc_ok) {
                // the dropped NodeClaim's pods get errors: if one of them is not pending, not all non-pending pods
                // scheduled (NONE); otherwise no new NodeClaim is left and the candidates' pods all landed: DELETE
                none = true;
                truncated_out = true;
            } else if (all_spot && has_spot) {  // computeSpotToSpotConsolidation
                if (!k.spot_to_spot) {
                    none = true;
                } else {
                    spot_only = true;  // Requirements.Add(capacity-type In [spot])
                    keep = my_t >= 0 && worst_launch_price(d, k, my_t, mt & k.spot_slots) < cprice;
                    const uint64_t km = ballot(keep);
                    int need = 0;
                    if (has_min && !min_values_ok(d, nch, nc_tmpl, my_t, km, lane, &need)) {
                        none = true;  // RemoveInstanceTypeOptionsByPriceAndMinValues keeps minValues
                    } else if (!km) {
                        none = true;
                    } else if (c1 - c0 == 1) {
                        // MinInstanceTypesForSpotToSpotConsolidation; the kept list is cut to max(15, minNeeded)
                        const int cut = has_min && need > 15 ? need : 15;
                        if (__popcll(km) < 15) none = true;
                        else keep = keep && __popcll(km & ((1ull << lane) - 1)) < cut;
                    }
                }
            } else {  // RemoveInstanceTypeOptionsByPriceAndMinValues
                keep = my_t >= 0 && worst_launch_price(d, k, my_t, mt, mr, mrw) < cprice;
                const uint64_t km = ballot(keep);
                if (!km || (has_min && !min_values_ok(d, nch, nc_tmpl, my_t, km, lane, nullptr))) none = true;
                spot_only = has_spot && has_od;  // spot/on-demand flexible replacement narrowed to spot
            }
            if (truncated_out && nc_nonpend == 0) {
                decision = KP_DECISION_DELETE;
                valid = 1;
            } else if (!none) {
                decision = KP_DECISION_REPLACE;
                const uint64_t ms = spot_only ? (mt & k.spot_slots) : mt;
                const double wl = keep ? worst_launch_price(d, k, my_t, ms, spot_only ? 0ull : mr, mrw) : DBL_MAX;
                if (!single) {  // filterOutSameInstanceType
                    double mp = DBL_MAX;
                    if (keep)
                        for (int c = c0; c < c1; c++)
                            if (k.cand_i[c * 4 + 2] == my_t && k.cand_price[c] < mp) mp = k.cand_price[c];
                    const double maxp = wave_min_f64(mp);
                    keep = keep && wl < maxp;
                }
                const uint64_t km = ballot(keep);
                valid = km != 0;
                nrep = __popcll(km);
                rprice = nrep ? wave_min_f64(keep ? wl : DBL_MAX) : 0.0;
                if (FULL && k.rec_i) {  // kp_consolidate_command: the replacement NodeClaim of this probe
                    const int nheld = RESV ? wave_sum_i32(lane < d.ro_ridw ? __popcll(nc_held) : 0) : 0;
                    if (keep) k.rec_i[4 + __popcll(km & ((1ull << lane) - 1))] = my_t;
                    if (lane == 0) {
                        k.rec_i[1] = nc_tmpl;
                        k.rec_i[2] = spot_only ? 1 : 0;
                        k.rec_i[3] = nrep;
                        k.rec_i[4 + 64] = nheld;
                    }
                    for (int kk = lane; kk < K; kk += 64) k.rec_hdr[kk] = nch[kk];
                    for (int i = lane; i < d.DW; i += 64) k.rec_words[i] = ncw[i];
                }
            }
        }
        if (FULL && k.rec_i && lane == 0) k.rec_i[0] = decision;
        if (prof) cy_dec = __builtin_amdgcn_s_memtime() - cd0;
        if (lane == 0) {
            kp_probe_result o;
            o.decision = decision;
            o.valid = valid;
            o.all_scheduled = (all && !(truncated_out && nc_nonpend > 0)) ? 1 : 0;
            o.n_new_nodeclaims = stop ? 2 : (truncated_out ? 0 : n_nc);
            o.n_replacement_types = nrep;
            o.n_pods = n;
            o.candidate_price = cprice;
            o.replacement_price = rprice;
            k.out[oi] = o;
            // counters stay in LDS until the worker exits (per-probe global atomics on 16 words serialise in L2)
            S.st[CS_POPS] += st_pops;
            S.st[CS_EX_NODES] += st_nodes;
            S.st[CS_NC_EVALS] += st_nc;
            S.st[CS_TMPL_EVALS] += st_tmpl;
            S.st[CS_PROBES] += 1;
            S.st[CS_BITMAP_WORDS] += st_words;
            S.st[CS_PLACED_EXISTING] += st_placed;
            S.st[CS_NEW_NC] += o.n_new_nodeclaims;
            S.st[CS_CHUNK_LOADS] += st_loads;
            S.st[CS_CACHE_HITS] += st_hits;
            S.st[CS_CHUNK_SKIPS] += st_skips;
            S.st[CS_RELAXED] += st_relax;
            if (MUT && mutp) S.st[CS_MUT] += 1;
            if (prof) {
                if (k.prof_probe) {
                    int64_t* pp = k.prof_probe + (size_t)oi * KP_CONS_PP;
                    pp[0] = cy_build;
                    pp[1] = cy_scan;
                    pp[2] = __builtin_amdgcn_s_memtime() - cy0;
                    pp[3] = n;
                    pp[4] = pf_load;
                    pp[5] = pf_prep;
                    pp[6] = pf_nodes;
                    pp[7] = pf_visits;
                    pp[8] = pf_many;
                    pp[9] = pf_iters;
                    pp[10] = pf_miss_cyc;
                    pp[11] = pf_miss;
                    pp[12] = cy_nc;
                    pp[13] = cy_dec;
                    pp[14] = st_loads;
                    pp[15] = st_skips;
                }
                S.st[CS_CYC_BUILD] += cy_build;
                S.st[CS_CYC_SCAN] += cy_scan;
                S.st[CS_CYC_NODECLAIM] += cy_nc;
                S.st[CS_CYC_DECIDE] += cy_dec;
                S.st[CS_CYC_TOTAL] += __builtin_amdgcn_s_memtime() - cy0;
            }
        }
        }
        __syncthreads();
    }
    if (lane < CS_COUNT && S.st[lane]) atomicAdd((unsigned long long*)&k.stats[lane], (unsigned long long)S.st[lane]);
}

// The fast variant takes its tables by value (kernel arguments).  The FULL variant takes them by pointer to device
// copies and reads them through const references (no per-lane scratch copy); an idle launch (the fast variant handed
// nothing over) exits at once.
template <bool FULL, bool RESV = false, bool TOPO = false, int NA = 0>
__global__ __launch_bounds__(64) void consolidate_kernel(KpDev d, KpCons k) {
    consolidate_body<FULL, RESV, TOPO, NA>(d, k);
}
template <bool RESV, bool TOPO, bool MUT = false>
__global__ __launch_bounds__(64) void consolidate_full_kernel(const KpDev* __restrict__ dp, const KpCons* __restrict__ kp) {
    if (kp->no_fast != 1 && ld32(&kp->next_probe[2]) == 0) return;
    consolidate_body<true, RESV, TOPO, 0, MUT, const KpDev&, const KpCons&>(*dp, *kp);
}

// cmax0[w][ai]: the largest headroom on active axis ai over the nodes of chunk w (one wave per chunk; lanes past E and
// axes past n_active hold INT64_MIN)
__global__ __launch_bounds__(64) void chunk_max_kernel(const int64_t* __restrict__ ex_head, int E, int A,
                                                        int64_t* __restrict__ cmax0) {
    const int w = blockIdx.x, j = w * 64 + threadIdx.x;
#pragma unroll
    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
        const int64_t h = (ai < A && j < E) ? ex_head[(size_t)ai * E + j] : INT64_MIN;
        const int64_t mx = wave_max64(h);
        if (threadIdx.x == 0) cmax0[(size_t)w * KP_LDS_AXES + ai] = mx;
    }
}

hipError_t kp_launch_cons_chunk_max(const KpDev& d, int64_t* cmax0, hipStream_t s) {
    if (d.E > 0) hipLaunchKernelGGL(chunk_max_kernel, dim3(d.EW), dim3(64), 0, s, d.ex_head, d.E, d.n_active, cmax0);
    return hipGetLastError();
}

// queue position of each pod: rank[queue0[i]] = i
__global__ void rank_kernel(const int32_t* __restrict__ queue0, int32_t* __restrict__ rank, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rank[queue0[i]] = i;
}
__global__ void pending_bits_kernel(const int32_t* __restrict__ pending, int n, const int32_t* __restrict__ rank,
                                    uint64_t* __restrict__ bits) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int r = rank[pending[i]];
        atomicOr((unsigned long long*)&bits[r >> 6], 1ull << (r & 63));
    }
}

// Dynamic LDS of consolidate_kernel: fixed block, NodeClaim digest, limits, candidate / modified-node bitmaps.
bool kp_cons_plan_lds(const KpDev& d, KpCons& k, int max_bytes) {
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t off = al(sizeof(ConsShared));
    k.off_hdr = (int)off;
    off = al(off + sizeof(ReqHdr) * (size_t)(d.K > 0 ? d.K : 1));
    k.off_words = (int)off;
    off = al(off + 8 * (size_t)(d.DW > 0 ? d.DW : 1));
    k.off_rem = (int)off;
    off = al(off + 8 * (size_t)(d.NT * d.R > 0 ? d.NT * d.R : 1));
    k.off_excl = (int)off;
    off = al(off + 8 * (size_t)(d.EW > 0 ? d.EW : 1));
    k.off_mod = (int)off;
    off = al(off + 8 * (size_t)(d.EW > 0 ? d.EW : 1));
    k.off_init = (int)off;
    off = al(off + 8 * (size_t)(d.EW > 0 ? d.EW : 1));
    k.off_rcap = (int)off;  // RESV: the probe's ReservationManager capacities (NewReservationManager per SimulateScheduling)
    off = al(off + (d.ro ? 4 * (size_t)(d.ro_nrid > 0 ? d.ro_nrid : 1) : 0));
    k.off_mutn = (int)off;  // MUT: nodes whose requirements the probe changed
    off = al(off + (k.mut ? 8 * (size_t)(d.EW > 0 ? d.EW : 1) : 0));
    k.off_xtc = (int)off;
    off = al(off + 8 * (size_t)(d.C < KP_CONS_XTC ? (d.C > 0 ? d.C : 1) : KP_CONS_XTC));
    k.off_touch = (int)off;  // TOPO: the probe's copied count rows and node host-count columns
    off = al(off + (k.G > 0 ? 8 * (size_t)((k.G + 63) / 64) : 0));
    k.off_hmod = (int)off;
    off = al(off + (k.G > 0 ? 8 * (size_t)(d.EW > 0 ? d.EW : 1) : 0));
    k.off_hpos = (int)off;  // TOPO: positive hostname domains per hostname-affinity group
    off = al(off + 4 * (size_t)(k.n_ha > 0 ? k.n_ha : 1));
    // the fast variant's store of the first chunks' headroom ([n_store][n_active][64] i64): up to KP_CONS_STORE chunks,
    // fewer when the cluster is smaller
    {
        const int A = d.n_active > 0 ? d.n_active : 1;
        int ns = d.EW < KP_CONS_STORE ? d.EW : KP_CONS_STORE;
        if (ns < 1) ns = 1;
        k.n_store = ns;
        k.off_hs = (int)off;
        off = al(off + (size_t)ns * A * 64 * 8);
    }
    // the chunk headroom summary, when it fits beside the rest (it is an accelerator, not needed for the result)
    k.off_cmax = (int)off;
    const size_t cm = 8 * (size_t)(d.EW > 0 ? d.EW : 1) * KP_LDS_AXES;
    k.use_cmax = (k.cmax0 != nullptr && d.E > 0 && off + cm <= (size_t)max_bytes) ? 1 : 0;
    if (k.use_cmax) off = al(off + cm);
    k.lds_bytes = (int)off;
    return (int)off <= max_bytes;
}

// Per-device kernel attributes, set by kp_ctx_create with the ctx's device current (see kp_ffd_set_attributes).
hipError_t kp_cons_set_attributes() {
    const void* fns[] = {(const void*)consolidate_kernel<false>, (const void*)consolidate_full_kernel<false, false>,
                         (const void*)consolidate_kernel<false, false, false, 1>,
                         (const void*)consolidate_kernel<false, false, false, 2>,
                         (const void*)consolidate_kernel<false, false, false, 3>,
                         (const void*)consolidate_kernel<false, false, false, 4>,
                         (const void*)consolidate_kernel<false, false, false, 5>,
                         (const void*)consolidate_kernel<false, false, false, 6>,
                         (const void*)consolidate_full_kernel<true, false>, (const void*)consolidate_kernel<false, false, true>,
                         (const void*)consolidate_full_kernel<false, true>, (const void*)consolidate_full_kernel<true, true>,
                         (const void*)consolidate_full_kernel<false, false, true>, (const void*)consolidate_full_kernel<true, false, true>,
                         (const void*)consolidate_full_kernel<false, true, true>, (const void*)consolidate_full_kernel<true, true, true>};
    for (const void* f : fns) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, KP_LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t kp_launch_consolidate(const KpDev& d, const KpCons& k, int n_workers, hipStream_t s, KpDev* d_dev,
                                 KpCons* d_k) {
    if (n_workers <= 0 || k.n_probes <= 0) return hipSuccess;
    const size_t lds = (size_t)k.lds_bytes;
    if (k.G > 0) {
        if (k.no_fast != 1) hipLaunchKernelGGL((consolidate_kernel<false, false, true>), dim3(n_workers), dim3(64), lds, s, d, k);
        if (k.no_fast != 2) {
            const dim3 gf(n_workers < KP_CONS_FULL_WORKERS ? n_workers : KP_CONS_FULL_WORKERS);  // as below
            if (k.mut) {  // MUT instantiation: per-probe node requirement copies
                if (d.ro) hipLaunchKernelGGL((consolidate_full_kernel<true, true, true>), gf, dim3(64), lds, s, d_dev, d_k);
                else hipLaunchKernelGGL((consolidate_full_kernel<false, true, true>), gf, dim3(64), lds, s, d_dev, d_k);
            } else if (d.ro) {
                hipLaunchKernelGGL((consolidate_full_kernel<true, true>), gf, dim3(64), lds, s, d_dev, d_k);
            } else {
                hipLaunchKernelGGL((consolidate_full_kernel<false, true>), gf, dim3(64), lds, s, d_dev, d_k);
            }
        }
        return hipGetLastError();
    }
    if (k.no_fast != 1) {
        const dim3 g(n_workers), b(64);
        switch (d.n_active) {
            case 1: hipLaunchKernelGGL((consolidate_kernel<false, false, false, 1>), g, b, lds, s, d, k); break;
            case 2: hipLaunchKernelGGL((consolidate_kernel<false, false, false, 2>), g, b, lds, s, d, k); break;
            case 3: hipLaunchKernelGGL((consolidate_kernel<false, false, false, 3>), g, b, lds, s, d, k); break;
            case 4: hipLaunchKernelGGL((consolidate_kernel<false, false, false, 4>), g, b, lds, s, d, k); break;
            case 5: hipLaunchKernelGGL((consolidate_kernel<false, false, false, 5>), g, b, lds, s, d, k); break;
            case 6: hipLaunchKernelGGL((consolidate_kernel<false, false, false, 6>), g, b, lds, s, d, k); break;
            default: hipLaunchKernelGGL(consolidate_kernel<false>, g, b, lds, s, d, k); break;
        }
    }
    if (k.no_fast != 2) {
        // the FULL variant runs one wave per SIMD (its registers): more workers than SIMDs only queue, and each worker,
        // even an idle one, first copies the kernel arguments to its scratch
        const dim3 gf(n_workers < KP_CONS_FULL_WORKERS ? n_workers : KP_CONS_FULL_WORKERS);
        if (k.mut) {
            if (d.ro) hipLaunchKernelGGL((consolidate_full_kernel<true, false, true>), gf, dim3(64), lds, s, d_dev, d_k);
            else hipLaunchKernelGGL((consolidate_full_kernel<false, false, true>), gf, dim3(64), lds, s, d_dev, d_k);
        } else if (d.ro) {
            hipLaunchKernelGGL((consolidate_full_kernel<true, false>), gf, dim3(64), lds, s, d_dev, d_k);
        } else {
            hipLaunchKernelGGL((consolidate_full_kernel<false, false>), gf, dim3(64), lds, s, d_dev, d_k);
        }
    }
    return hipGetLastError();
}

// The multi-node probes' pods in queue order, built once per call: the pods of candidates [0, nu) (every multi-node
// prefix of the call draws from them) and the pending pods, one entry per queue position holding either, as
// {pod | pending << 31, candidate index or -1 for a pending pod}.  A probe over candidates [0, c1) takes the entries
// with index < c1 in order (consolidate_kernel), instead of marking and scanning a bitmap over every queue position.
// One block: mark the union's queue positions (and each position's candidate), then compact the marked positions.
__global__ __launch_bounds__(1024) void multi_union_kernel(const int32_t* __restrict__ cand_off,
                                                           const int32_t* __restrict__ cand_pods,
                                                           const int32_t* __restrict__ rank,
                                                           const int32_t* __restrict__ queue0,
                                                           const uint64_t* __restrict__ pend_bits, int n_pending, int PW,
                                                           int nu, uint64_t* __restrict__ ubits,
                                                           int32_t* __restrict__ rcand, int2* __restrict__ ulist,
                                                           int32_t* __restrict__ ulen) {
    __shared__ int32_t wsum[1024];
    __shared__ int32_t carry;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int w = tid; w < PW; w += nt) ubits[w] = 0;
    if (tid == 0) carry = 0;
    __syncthreads();
    // candidate of CSR entry i: the last c with cand_off[c] <= i (binary search over the union's candidates)
    const int e0 = cand_off[0], e1 = cand_off[nu];
    for (int i = e0 + tid; i < e1; i += nt) {
        int lo = 0, hi = nu - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cand_off[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const int r = rank[cand_pods[i]];
        atomicOr((unsigned long long*)&ubits[r >> 6], 1ull << (r & 63));
        rcand[r] = lo;
    }
    __syncthreads();
    for (int wb = 0; wb < PW; wb += nt) {
        const int w = wb + tid;
        const uint64_t mine = w < PW ? ubits[w] : 0ull;
        const uint64_t pend = (w < PW && n_pending) ? pend_bits[w] : 0ull;
        uint64_t x = mine | pend;
        const int cnt = __popcll(x);
        wsum[tid] = cnt;
        __syncthreads();
        for (int o = 1; o < nt; o <<= 1) {  // inclusive scan of the words' counts
            const int v = tid >= o ? wsum[tid - o] : 0;
            __syncthreads();
            wsum[tid] += v;
            __syncthreads();
        }
        int pos = carry + wsum[tid] - cnt;
        while (x) {
            const int b = __ffsll((unsigned long long)x) - 1;
            x &= x - 1;
            const int r = w * 64 + b;
            const bool pd = (pend >> b) & 1ull;
            ulist[pos++] = make_int2(queue0[r] | (int32_t)((uint32_t)pd << 31), pd ? -1 : rcand[r]);
        }
        __syncthreads();
        if (tid == nt - 1) carry += wsum[tid];
        __syncthreads();
    }
    if (tid == 0) ulen[0] = carry;
}

hipError_t kp_launch_multi_union(const KpCons& k, int nu, uint64_t* ubits, int32_t* rcand, int2* ulist, int32_t* ulen,
                                 const int32_t* queue0, hipStream_t s) {
    hipLaunchKernelGGL(multi_union_kernel, dim3(1), dim3(1024), 0, s, k.cand_off, k.cand_pods, k.rank, queue0,
                       k.pend_bits, k.n_pending, k.PW, nu, ubits, rcand, ulist, ulen);
    return hipGetLastError();
}

hipError_t kp_launch_cons_prep(const int32_t* queue0, int P, int32_t* rank, const int32_t* pending, int n_pending,
                               uint64_t* pend_bits, hipStream_t s) {
    if (P > 0) hipLaunchKernelGGL(rank_kernel, dim3((P + 255) / 256), dim3(256), 0, s, queue0, rank, P);
    if (n_pending > 0)
        hipLaunchKernelGGL(pending_bits_kernel, dim3((n_pending + 255) / 256), dim3(256), 0, s, pending, n_pending,
                           rank, pend_bits);
    return hipGetLastError();
}
