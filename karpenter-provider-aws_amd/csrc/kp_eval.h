// kp_eval.h — NodeClaim.Add evaluated by ONE wave (64 lanes), LDS-resident operands.
//
// Reference semantics ([core] sigs.k8s.io/karpenter pkg/controllers/provisioning/scheduling/nodeclaim.go):
//   NodeClaim.Add(pod):
//     Taints(template).ToleratesPod(pod)
//     nodeClaimRequirements.Compatible(podRequirements, AllowUndefinedWellKnownLabels); Add(podRequirements)
//     requests = Merge(nodeClaim.requests, pod.requests)
//     remaining = filterInstanceTypesByRequirements(options, reqs, requests):
//         it.Requirements.Intersects(reqs) ∧ resources.Fits(requests, it.Allocatable()) ∧
//         ∃ offering: Available ∧ reqs.IsCompatible(offering.Requirements, AllowUndefinedWellKnownLabels)
//         then SatisfiesMinValues (MIN_VALUES_POLICY=Strict)
//
// Encoding that makes this a bitset sweep:
//   * options ⊆ compatible(nodeClaim requirements) is an invariant, and for a single-valued label
//     Has(merged, v) = Has(nc, v) ∧ Has(class, v); so label compatibility of a type reduces to the class's
//     precomputed V bitset, except for types whose label is DoesNotExist, which survive only when the merged
//     operator is NotIn/DoesNotExist (dne masks), and multi-valued labels (zone, capacity-type, ...), tested per
//     type as (type value mask ∧ merged admissible mask) ≠ 0;
//   * offerings reduce to one u64 per type over (zone × capacity-type) slots; the merged requirements give the
//     admissible slot mask;
//   * Fits compares the request totals with LDS-staged allocatable columns of the active resource axes.
#pragma once
#include "kp_wave.h"
#include "kp_device.h"

// wave-count namespace (kp_layout.h KP_WNS): the 4-wave topology units and the 8-wave units hold distinct
// definitions of the wave-shaped types (FfdShared, TeamBuf ...) and of every helper that uses them
namespace KP_WNS {

// Per-wave LDS scratch: merged requirements of the class's keys, resulting options, minValues bitset.
struct WaveScratch {
    ReqHdr hdr[KP_MAX_CLASS_KEYS];
    uint64_t words[KP_MAX_SCR_WORDS];
    uint64_t opts[KP_TW_MAX];
    uint64_t minbits[KP_MAX_MIN_WORDS];  // minValues distinct values; after the reservation step of a successful Add:
                                         // the reservations the NodeClaim holds (ResvTab::ridw words)
    int32_t hr[KP_LDS_AXES];   // quick-accept headroom of the chosen witness type (scaled, lower bound)
    int32_t memo_ok;           // a failed evaluation may be memoised for the shape (it did not depend on topology
                               // counts: see topo_narrow; one that depended on reservation capacity is memoised
                               // until a capacity comes back from 0, see the reservation step)
    int32_t rlive;             // success: the new options keep a compatible available reserved offering
    // success under MIN_VALUES_POLICY=BestEffort: keys whose minValues the Add relaxes to the distinct values the
    // remaining options offer (SatisfiesMinValues' unsatisfiable keys); the commit writes them into the NodeClaim
    int32_t n_minrel;
    int32_t minrel_k[KP_MAX_CLASS_KEYS];
    int32_t minrel_v[KP_MAX_CLASS_KEYS];
};

// An unmet minValues key: Strict fails the Add; BestEffort records the relaxation (wave-uniform).
__device__ __forceinline__ bool min_values_unmet(const KpDev& d, WaveScratch& ws, int k, int count, int lane) {
    if (!d.best_effort) return false;
    if (lane == 0 && ws.n_minrel < KP_MAX_CLASS_KEYS) {
        ws.minrel_k[ws.n_minrel] = k;
        ws.minrel_v[ws.n_minrel] = count;
        ws.n_minrel++;
    }
    return true;
}

// Apply an Add's BestEffort minValues relaxations to NodeClaim slot n (after commit_reqs).
__device__ __forceinline__ void commit_min_relax(const KpDev& d, const WaveScratch& ws, int n, int lane) {
    if (lane < ws.n_minrel) d.nc_hdr[(size_t)n * d.K + ws.minrel_k[lane]].minv = ws.minrel_v[lane];
}

// Class-side operands of the evaluation, cached in LDS while consecutive pods share a class.
struct ClassCache {
    int cls;
    int nck;
    uint64_t tol;
    uint32_t flags;
    int role[5];  // class-key index of zone, capacity-type, zone-id, reservation-id, reservation-type (or -1)
    int key[KP_MAX_CLASS_KEYS];
    int wsoff[KP_MAX_CLASS_KEYS];
    int nw[KP_MAX_CLASS_KEYS];
    int woff[KP_MAX_CLASS_KEYS];
    uint32_t kflags[KP_MAX_CLASS_KEYS];
    int kcat[KP_MAX_CLASS_KEYS];
    int kmulti[KP_MAX_CLASS_KEYS];
    int nval[KP_MAX_CLASS_KEYS];
    int nbB[KP_MAX_CLASS_KEYS];
    ReqHdr hdr[KP_MAX_CLASS_KEYS];
    uint64_t words[KP_MAX_SCR_WORDS];
    uint64_t V[KP_TW_MAX];
    uint64_t dne[KP_MAX_CLASS_KEYS][KP_DNE_TW];
    uint32_t kneutral;          // class keys present only for topology narrowing (bit per class-key index)
    int ntc, ntr;               // topology groups constraining / recording the class
    int tc[KP_CC_TC];           // the first KP_CC_TC constraining groups: group | self << 30 (the others: cls_tc)
    int tc_ki[KP_CC_TC];        // class-key index of a value-keyed group's key (-1 for hostname groups)
    int tr[KP_CC_REC];          // the first KP_CC_REC recording groups (the others: rec_entry)
    int tr_ki[KP_CC_REC];       // class-key index of the group's key, -1 when the class does not constrain it
};

// Offering-role keys (zone, capacity-type, zone-id, reservation-id, reservation-type) of the solve.
struct Roles {
    int key[5];
    int woff[5];
    int nw[5];
};

// Topology counts of one consolidation probe (SimulateScheduling builds its own Topology: the domain groups, then
// countDomains over the bound pods minus the ones it reschedules).  The prepared pass holds the base counts of every bound
// pod (d.tg_cnt / d.tg_hcnt, read-only in probes); a probe keeps its own value-keyed rows (copied from the base on first
// use, the probe's candidates' pods subtracted at probe start) and hostname-count deltas per node column (valid once the
// node's hmod bit is set; column E is the probe's in-flight NodeClaim).  Hostname pod affinity (whose bootstrap counts
// domains) keeps the probe's positive-domain count per group (hpos).
struct ProbeTopo {
    int32_t* cnt;          // [G][64] value-keyed counts (row g valid when touched bit g is set)
    uint64_t* known;       // [G] registered domains of row g
    uint64_t* touched;     // LDS [ceil(G / 64)]
    int32_t* hd;           // [HG][E + 1] hostname-count deltas
    uint64_t* hmod;        // LDS [EW]: node column valid
    const uint64_t* dgk;   // [G] domains of buildDomainGroups (registered before any pod is counted)
    int32_t* hpos;         // LDS [n_ha]: hostname domains holding a selected pod, per hostname-affinity group
    const int32_t* ha;     // [G] hostname-affinity group index into hpos, or -1
    uint64_t* born;        // LDS: the probe's born late identities (KpDev.tg_late)
    const uint64_t* excl;  // LDS [EW]: the probe's candidates (their nodes leave the cluster)
    int E, HG;
};

// Per-pod snapshot of the value-keyed topology groups that constrain the current pod's class (FFD kernel, LDS; filled by
// topo_prefilter_setup in CC.tc order): counts only change when a pod commits, so every candidate evaluation of the pod
// reads them here instead of from the global counters.
// One row per group; the LDS plan holds KpDev.snap_rows of them (the most constraining groups of any class, <=
// KP_SNAP_ROWS), so a solve pays only for the rows its classes use.
struct SnapRow {
    int32_t cnt[64];   // domain counts (0 where the domain is not registered)
    uint8_t rk[64];    // value-name rank of each domain (tie-break)
    uint64_t known;    // registered domains
    uint64_t podhas;   // domains the pod's own requirement for the key admits
};
struct TopoSnap {
    SnapRow r[KP_SNAP_ROWS];
};

// Tables shared by every evaluation of a kernel (LDS in ffd_kernel).
struct EvalEnv {
    const int64_t* alloc;      // [lds_nstage][astride] staged allocatable of the first active axes
    const uint64_t* avail;     // [T] available od/spot slot mask per type
    const uint16_t* multi16;   // [n_multi][astride] multi-valued label masks, or null → global multi_mask
    int astride;               // row stride of alloc / multi16
    const int* slot_zone;
    const int* slot_ct;
    const int* slot_zoneid;
    const Roles* roles;
    uint64_t min_tmpl_mask;    // templates whose requirements carry minValues
    const ResvTab* ro;         // reserved offerings (null: none)
    const uint32_t* type_ro;   // [T] the type's reserved-offering rows (packed, ro_span_bits)
    const int32_t* rcap;       // ReservationManager capacity by reservation (ResvTab::rid; LDS)
    int resv_on;               // run the reservation step of NodeClaim.Add
    const ProbeTopo* pt;       // consolidation probe topology counts (eval_wave<..., CT = true>)
    const TopoSnap* snap;      // FFD kernel: the current pod's topology snapshot (null: read the global counters)
};

// Cooperative fill by all threads of the block; contains two __syncthreads().
// Topology.Update of a pod relaxed into a class that owns the late bits `add`: each group is created unless a variant
// sibling of its identity already was (the identity's group then exists, with that sibling's semantics).
__device__ __forceinline__ uint64_t topo_birth(const KpDev& d, uint64_t born, uint64_t add) {
    if (!d.late_sib) return born | add;
    for (uint64_t x = add & ~born; x; x &= x - 1) {
        const int b = __ffsll((unsigned long long)x) - 1;
        if (!(born & d.late_sib[b])) born |= 1ull << b;
    }
    return born;
}
// A class's constraint on group g: for a variant group, the identity's born variant (g itself until one is born).
__device__ __forceinline__ int topo_variant(const KpDev& d, int g, uint64_t born) {
    if (!d.late_sib) return g;
    const int lt = d.tg_late[g];
    if (lt < 0) return g;
    const uint64_t m = born & d.late_sib[lt];
    return m ? d.late_grp[__ffsll((unsigned long long)m) - 1] : g;
}

// born: the late topology groups created so far (routes a constraint on a variant group to the born variant).  TOPO:
// the caller's instantiation has topology groups (without, their lists are not filled: G = 0)
template <bool TOPO = false>
__device__ inline void fill_class_cache(const KpDev& d, int c, ClassCache& CC, int tid, int nthr, uint64_t born = 0) {
    const int k0 = d.cls_koff[c], nck = d.cls_koff[c + 1] - k0;
    for (int i = tid; i < nck; i += nthr) {
        const int k = d.cls_keys[k0 + i];
        CC.key[i] = k;
        CC.wsoff[i] = d.cls_wsoff[k0 + i];
        CC.nw[i] = d.nw[k];
        CC.woff[i] = d.woff[k];
        CC.kflags[i] = d.kflags[k];
        CC.kcat[i] = d.kcat[k];
        CC.kmulti[i] = d.kmulti[k];
        CC.nval[i] = d.nval[k];
        CC.hdr[i] = d.cls_hdr[(size_t)c * d.K + k];
        int nb = 0;
        for (int w = 0; w < d.nw[k]; w++) {
            const uint64_t x = d.cls_words[(size_t)c * d.DW + d.woff[k] + w];
            CC.words[d.cls_wsoff[k0 + i] + w] = x;
            nb += __popcll(x);
        }
        CC.nbB[i] = nb;
        const int kc = d.kcat[k];
        for (int w = 0; w < d.TW && w < KP_DNE_TW; w++) CC.dne[i][w] = kc >= 0 ? d.dne_mask[(size_t)kc * d.TW + w] : 0ull;
    }
    for (int w = tid; w < d.TW; w += nthr) CC.V[w] = d.V[(size_t)c * d.TW + w];
    if (tid == 0) {
        CC.cls = c;
        CC.nck = nck;
        CC.tol = c < d.C ? d.tol[c] : ~0ull;
        CC.flags = d.cls_flags[c];
        uint32_t kn = 0;
        if (d.cls_kneutral)
            for (int i = 0; i < nck; i++) kn |= d.cls_kneutral[k0 + i] ? (1u << i) : 0u;
        CC.kneutral = kn;
        CC.ntc = (TOPO && c < d.C && d.G > 0) ? d.cls_tcoff[c + 1] - d.cls_tcoff[c] : 0;
        CC.ntr = (TOPO && c < d.C && d.G > 0) ? d.cls_troff[c + 1] - d.cls_troff[c] : 0;
    }
    __syncthreads();
    if (tid < 5) {
        const int rk = tid == 0 ? d.key_zone : tid == 1 ? d.key_ct : tid == 2 ? d.key_zoneid : tid == 3 ? d.key_resvid : d.key_resvtype;
        int idx = -1;
        for (int i = 0; i < nck; i++)
            if (CC.key[i] == rk && rk >= 0) idx = i;
        CC.role[tid] = idx;
    }
    // topology group lists with the class-key index of each group's key
    if (TOPO && tid < CC.ntc + CC.ntr) {
        const bool cons = tid < CC.ntc;
        const int e = cons ? d.cls_tc[d.cls_tcoff[c] + tid] : d.cls_tr[d.cls_troff[c] + tid - CC.ntc];
        const int4 info = d.tg_info[e & 0x3FFFFFFF];
        int ki = -1;
        if (!(info.x & TG_HOST))
            for (int i = 0; i < nck; i++)
                if (CC.key[i] == info.y) ki = i;
        if (cons) {
            if (tid < KP_CC_TC) {
                CC.tc[tid] = (e & ~0x3FFFFFFF) | topo_variant(d, e & 0x3FFFFFFF, born);
                CC.tc_ki[tid] = ki;
            }
        } else if (tid - CC.ntc < KP_CC_REC) {
            CC.tr[tid - CC.ntc] = e;
            CC.tr_ki[tid - CC.ntc] = ki;
        }
    }
    __syncthreads();
}

// NodeClaim request totals are updated with device-scope atomics by the quick-accept path; read them past L1.
__device__ __forceinline__ int64_t ld_req(const int64_t* p) {
    return __hip_atomic_load(const_cast<int64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
    return wave_reduce64(x, [](uint64_t a, uint64_t b) { return a | b; });
}
__device__ __forceinline__ int64_t wave_max64(int64_t x) {
    return (int64_t)wave_reduce64((uint64_t)x, [](uint64_t a, uint64_t b) { return (int64_t)b > (int64_t)a ? b : a; });
}

// Has(merged, v) for an offering-role key r: merged = scratch (class constrains the key) or the base digest.
__device__ __forceinline__ bool role_adm(const KpDev& d, const EvalEnv& E, const ClassCache& CC, const WaveScratch& ws,
                                         const ReqHdr* Ahdr, const uint64_t* Aw, int r, int v) {
    const int k = E.roles->key[r];
    if (k < 0) return true;
    const int i = CC.role[r];
    if (i >= 0) return req_has(d, k, v, ws.hdr[i], ws.words + CC.wsoff[i]);
    const ReqHdr h = Ahdr[k];
    if (!(h.flags & RF_DEF)) return true;  // undefined well-known offering key → AllowUndefined
    return req_has(d, k, v, h, Aw + E.roles->woff[r]);
}
// Offering carries the key as DoesNotExist: passes iff the merged operator is NotIn / DoesNotExist.
__device__ __forceinline__ bool role_dneok(const KpDev& d, const EvalEnv& E, const ClassCache& CC,
                                           const WaveScratch& ws, const ReqHdr* Ahdr, const uint64_t* Aw, int r) {
    const int k = E.roles->key[r];
    if (k < 0) return true;
    const int i = CC.role[r];
    ReqHdr h;
    const uint64_t* w;
    int n = E.roles->nw[r];
    if (i >= 0) {
        h = ws.hdr[i];
        w = ws.words + CC.wsoff[i];
    } else {
        h = Ahdr[k];
        if (!(h.flags & RF_DEF)) return true;
        w = Aw + E.roles->woff[r];
    }
    return op_notin_or_dne(req_op(h.flags, popc_words(w, n)));
}

// Offerings.Available() ∧ reqs.IsCompatible(offering.Requirements) for the reserved offerings: capacity-type In
// [reserved], zone, zone-id, reservation-id In [id], reservation-type In [type] (offering.go:178-186).  64 rows per
// ballot; lane q returns word q of the row bitset.
__device__ __forceinline__ uint64_t resv_adm(const KpDev& d, const EvalEnv& E, const ClassCache& CC, const WaveScratch& ws,
                                             const ReqHdr* Ahdr, const uint64_t* Aw, int lane) {
    const ResvTab& X = *E.ro;
    uint64_t mine = 0;
    for (int q = 0; q < X.w; q++) {
        const int i = q * 64 + lane;
        bool ok = false;
        if (i < X.n && ((X.avail[q] >> lane) & 1ull)) {
            const int zid = X.zid[i], rt = X.rtype[i];
            ok = X.type[i] >= 0 && role_adm(d, E, CC, ws, Ahdr, Aw, 1, X.ctv) && role_adm(d, E, CC, ws, Ahdr, Aw, 0, X.zone[i]) &&
                 (zid < 0 || role_adm(d, E, CC, ws, Ahdr, Aw, 2, zid)) && role_adm(d, E, CC, ws, Ahdr, Aw, 3, X.ridv[i]) &&
                 (rt < 0 ? role_dneok(d, E, CC, ws, Ahdr, Aw, 4) : role_adm(d, E, CC, ws, Ahdr, Aw, 4, rt));
        }
        const uint64_t m = ballot(ok);
        if (lane == q) mine = m;
    }
    return mine;
}

// Quick-accept witness for the NodeClaim state an evaluation produces (options `newword`, totals `tot`).
// Lazy Fits: request totals only grow, so filterInstanceTypesByRequirements' Fits term applied at every Add equals
// Fits against the final totals; a NodeClaim whose absorbed class repeats accepts the pod iff SOME option still fits.
// One fitting option (the witness) proves acceptance.  The witness maximises the number of further copies of the
// current pod that fit (scored inside the type sweep, from the allocatable values it already loaded);
// ws.hr[a] = floor((alloc[a][w] - tot[a]) >> qshift[a]) is a lower bound of its headroom that the quick path
// decrements by ceil(pod[a] >> qshift[a]) per accepted pod.  minValues templates need the full
// option set, so they get hr = -1 (never quick).
struct WitnessAcc {
    float inv[KP_LDS_AXES];
    float best;
    int bt;
    bool on;
    __device__ __forceinline__ void init(const KpDev& d, const EvalEnv& E, const int64_t* pod_req) {
        on = d.lds_A > 0 && E.alloc && pod_req;
        best = -1.0f;
        bt = 0x7fffffff;
#pragma unroll
        for (int ai = 0; ai < KP_LDS_AXES; ai++) {
            const int64_t p = (on && ai < d.lds_A) ? pod_req[d.active_axes[ai]] : 0;
            inv[ai] = p > 0 ? 1.0f / (float)p : 0.0f;
        }
    }
    // lane's type t survived with staged allocatable av[] against totals tot[]
    __device__ __forceinline__ void add(const int64_t* av, const int64_t* tot, int t) {
        float sc = 3.0e38f;
#pragma unroll
        for (int ai = 0; ai < KP_LDS_AXES; ai++)
            // i64 → f64 → f32: four VALU ops instead of the expanded i64 → f32 sequence (the score is a heuristic)
            if (inv[ai] > 0.0f) sc = fminf(sc, (float)(double)(av[ai] - tot[ai]) * inv[ai]);
        if (sc > best) {
            best = sc;
            bt = t;
        }
    }
    __device__ __forceinline__ void take(float ob, int ot) {
        if (ob > best || (ob == best && ot < bt)) {
            best = ob;
            bt = ot;
        }
    }
    // arg-best over the wave ((score desc, type asc) is a total order, so the reduction tree does not matter); every
    // lane ends with the wave's best
    __device__ __forceinline__ void reduce_wave() {
        KP_ASSERT_FULL_WAVE();
        take(__uint_as_float(dpp32<kDppQuadXor1>(__float_as_uint(best))), (int)dpp32<kDppQuadXor1>((uint32_t)bt));
        take(__uint_as_float(dpp32<kDppQuadXor2>(__float_as_uint(best))), (int)dpp32<kDppQuadXor2>((uint32_t)bt));
        take(__uint_as_float(dpp32<kDppRowHalfMirror>(__float_as_uint(best))), (int)dpp32<kDppRowHalfMirror>((uint32_t)bt));
        take(__uint_as_float(dpp32<kDppRowMirror>(__float_as_uint(best))), (int)dpp32<kDppRowMirror>((uint32_t)bt));
        {
            const float b0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best), 0));
            const int t0 = __builtin_amdgcn_readlane(bt, 0);
            const float b1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best), 16));
            const int t1 = __builtin_amdgcn_readlane(bt, 16);
            const float b2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best), 32));
            const int t2 = __builtin_amdgcn_readlane(bt, 32);
            const float b3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best), 48));
            const int t3 = __builtin_amdgcn_readlane(bt, 48);
            best = b0;
            bt = t0;
            take(b1, t1);
            take(b2, t2);
            take(b3, t3);
        }
    }
    // ws.hr from the arg-best (reduced: already wave- or team-reduced)
    __device__ __forceinline__ void finish(const KpDev& d, const EvalEnv& E, const int64_t* tot, bool minv,
                                           WaveScratch& ws, int lane, bool reduced = false) {
        const int A = d.lds_A;
        if (A == 0) return;
        if (!on || minv) {
            if (lane < A) ws.hr[lane] = -1;
            return;
        }
        if (!reduced) reduce_wave();
        int64_t my = 0;
#pragma unroll
        for (int ai = 0; ai < KP_LDS_AXES; ai++)
            if (lane == ai) my = tot[ai];
        if (lane < A) {
            const int64_t h = E.alloc[lane * E.astride + bt] - my;
            ws.hr[lane] = h < 0 ? -1 : (int32_t)(h >> qshift_of(d, lane));
        }
    }
};

// One evaluation shared by every wave of the block (TEAM): each wave sweeps the option words w ≡ rank (mod n); the
// partial results meet here (double-buffered by the parity of the joins actually reached — eval_wave's `joins`, which
// every wave of the block counts alike since they take the same early rejects — so one barrier per evaluation suffices).
struct TeamBuf {
    uint64_t nw[KP_TW_MAX];    // remaining options, by word (written by the word's wave)
    uint64_t any[KP_NWAVES];   // per wave: OR of its words
    float best[KP_NWAVES];     // per wave: witness arg-best (score, type)
    int bt[KP_NWAVES];
};

struct EvalIn {
    const ReqHdr* Ahdr;       // base requirements digest (NodeClaim, template or empty)
    const uint64_t* Aw;
    uint64_t opts;            // lane l < TW: option word l
    const int64_t* base_req;  // [R] (global) or null
    const int64_t* pod_req;   // [R] (LDS or global) or null
    int tmpl;                 // template of the NodeClaim (taints bit, minValues keys)
    bool compat;              // taints + Requirements.Compatible
    bool force_off;           // always apply the offering test (template filter)
    long long* prof;          // LDS stage-cycle counters (diagnostics) or null
    int host;                 // topology hostname domain of the candidate (E + NodeClaim id)
    uint64_t held;            // lane r < ResvTab::ridw: word r of the reservations the candidate holds (0: new NodeClaim)
};

__device__ __forceinline__ int ld_i32(const int32_t* p) {
    return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_u64(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    return wave_reduce32(x, [](uint32_t a, uint32_t b) { return b < a ? b : a; });
}
__device__ __forceinline__ int wave_min_i32(int x) {
    return (int)wave_reduce32((uint32_t)x, [](uint32_t a, uint32_t b) { return (int)b < (int)a ? b : a; });
}

// ---- probe topology counts (ProbeTopo) ----
// Row g of the probe's value-keyed counts: base - dec (the probe's candidates' pods, at probe start) or the base (first
// use); its registered domains are buildDomainGroups' plus every domain with a positive count.  Hostname rows: column
// j < E is node j, column E the probe's in-flight NodeClaim, E + 1 a NodeClaim being created (no pods yet).
__device__ inline void pt_init_row(const KpDev& d, const ProbeTopo& P, int g, const int32_t* dec, int lane) {
    const int32_t v = d.tg_cnt[(size_t)g * 64 + lane] - (dec ? dec[lane] : 0);
    __hip_atomic_store(&P.cnt[(size_t)g * 64 + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t kn = P.dgk[g] | ballot(v > 0);
    if (lane == 0) {
        __hip_atomic_store(&P.known[g], kn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        P.touched[g >> 6] |= 1ull << (g & 63);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void pt_row(const KpDev& d, const ProbeTopo& P, int g, int lane) {
    const uint64_t t = __builtin_amdgcn_readfirstlane((int)(uint32_t)(P.touched[g >> 6] >> (g & 63))) & 1;
    if (!t) pt_init_row(d, P, g, nullptr, lane);
}
__device__ __forceinline__ int pt_hcnt(const KpDev& d, const ProbeTopo& P, int hrow, int host) {
    int32_t* col = P.hd + (size_t)hrow * (P.E + 1);
    if (host > P.E) return 0;  // a NodeClaim not created yet
    if (host == P.E) return ld_i32(col + P.E);
    int c = d.tg_hcnt[(size_t)hrow * d.HN + host];
    if ((P.hmod[host >> 6] >> (host & 63)) & 1ull) c += ld_i32(col + host);
    return c;
}
// nextDomainAffinity's bootstrap test for a self-selecting hostname affinity (entry T of the class, group g): no host
// the pod's domains admit holds a selected pod (options.Len() == 0).  podDomains is every host unless the pod requires
// the hostname (T.hdom): In — none of the listed existing nodes is positive; NotIn — every positive host is listed.
// A listed node among a consolidation probe's candidates counts what its own reschedulable pods leave.  Whole wave.
template <bool CT>
__device__ inline bool host_aff_unseeded(const KpDev& d, const KpTopoCons& T, int g, const ProbeTopo* pt, int lane) {
    const int pos = CT ? pt->hpos[pt->ha[g]] : ld_i32(&d.tg_pos[g]);
    const int mode = T.hdom & 3;
    if (mode == 0) return pos == 0;
    const int n = T.hdom >> 2, hrow = -1 - T.key;
    int np = 0;
    for (int b = 0; b < n; b += 64) {
        bool p = false;
        if (b + lane < n) {
            const int2 h = d.tce_hosts[T.podhas + b + lane];
            if (CT && ((pt->excl[h.x >> 6] >> (h.x & 63)) & 1ull)) p = h.y != 0;
            else p = (CT ? pt_hcnt(d, *pt, hrow, h.x) : ld_i32(&d.tg_hcnt[(size_t)hrow * d.HN + h.x])) > 0;
        }
        np += __popcll(ballot(p));
    }
    return mode == 1 ? np == 0 : pos == np;
}

// one more pod counted in hostname row hrow at `host` (whole wave)
__device__ inline void pt_hadd(const ProbeTopo& P, int hrow, int host, int lane) {
    if (host < P.E && !((P.hmod[host >> 6] >> (host & 63)) & 1ull)) {
        for (int r = lane; r < P.HG; r += 64)
            __hip_atomic_store(&P.hd[(size_t)r * (P.E + 1) + host], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) P.hmod[host >> 6] |= 1ull << (host & 63);
    }
    if (lane == 0) atomicAdd(&P.hd[(size_t)hrow * (P.E + 1) + host], 1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// Topology.AddRequirements ([core] scheduling/topology.go) for one candidate, after the requirement merge: every group
// that constrains the pod's class yields its allowed domains (TopologyGroup.Get: nextDomainTopologySpread /
// nextDomainAffinity / nextDomainAntiAffinity), all computed from the same merged requirements (nodeDomains) and
// intersected per key, then Compatible(nodeClaimRequirements, topologyRequirements) and Add narrow the scratch.
// Value-keyed groups: lane v examines value id v of the key (<= 64 values).  Go picks among equal counts by map
// iteration order; the smallest value name (vrank) is the canonical choice (oracle/orc_solve.cpp topo_get).
// Hostname groups: the candidate's own host is the only domain its requirements allow (hostname In [host]).
// ws.memo_ok is cleared when the outcome depends on counts (a count check failed or a key was narrowed).
// CT: the counts are a consolidation probe's (pt).
template <bool CT = false>
__device__ __forceinline__ bool topo_narrow(const KpDev& d, const ClassCache& CC, WaveScratch& ws, int host, bool allow_wk,
                                         int lane, const ProbeTopo* pt = nullptr, const TopoSnap* snap = nullptr) {
    int nk = 0;
    int kidx[KP_MAX_TOPO_KEYS];
    uint64_t kmask[KP_MAX_TOPO_KEYS];
    for (int e = 0; e < CC.ntc; e++) {
        // beyond the cached entries: the class's list (no variant groups there, kp_solve_prepare), the key's class index
        const int te = e < KP_CC_TC ? CC.tc[e] : d.cls_tc[d.cls_tcoff[CC.cls] + e];
        const int g = te & 0x3FFFFFFF, self = (te >> 30) & 1;
        const int4 info = d.tg_info[g];
        int ki = -1;
        if (e < KP_CC_TC) {
            ki = CC.tc_ki[e];
        } else if (!(info.x & TG_HOST)) {
            for (int i = 0; i < CC.nck; i++)
                if (CC.key[i] == info.y) ki = i;
        }
        const int type = info.x & TG_TYPE;
        if (info.x & TG_HOST) {
            const int cnt = CT ? pt_hcnt(d, *pt, d.tg_hrow[g], host) : ld_i32(&d.tg_hcnt[(size_t)d.tg_hrow[g] * d.HN + host]);
            bool ok;
            if (type == 0) ok = cnt + self <= info.z;             // spread: hostname domainMinCount is 0
            else if (type == 2) ok = cnt == 0;                    // anti-affinity: an empty domain
            else ok = cnt > 0 || (self && host_aff_unseeded<CT>(d, d.cls_tce[d.cls_tcoff[CC.cls] + e], g, pt, lane));  // affinity (self-selecting bootstrap)
            if (!ok) {
                ws.memo_ok = 0;
                return false;
            }
            continue;
        }
        const int k = info.y;
        const bool valid = lane < CC.nval[ki];
        bool kn, pod_has;
        int cnt;
        uint32_t rk;
        if (!CT && snap && CC.ntc <= KP_SNAP_ROWS) {
            kn = valid && ((snap->r[e].known >> lane) & 1ull);
            cnt = kn ? snap->r[e].cnt[lane] : 0;
            pod_has = valid && ((snap->r[e].podhas >> lane) & 1ull);
            rk = valid ? snap->r[e].rk[lane] : 0xFFu;
        } else {
            if (CT) pt_row(d, *pt, g, lane);
            const uint64_t known = ld_u64(CT ? &pt->known[g] : &d.tg_known[g]);
            kn = valid && ((known >> lane) & 1ull);
            cnt = kn ? ld_i32(CT ? &pt->cnt[(size_t)g * 64 + lane] : &d.tg_cnt[(size_t)g * 64 + lane]) : 0;
            // podDomains: the class's strict requirements (KpTopoCons)
            pod_has = valid && ((d.cls_tce[d.cls_tcoff[CC.cls] + e].podhas >> lane) & 1ull);
            rk = valid ? d.vrank[(size_t)k * 64 + lane] : 0xFFu;
        }
        const ReqHdr nh = ws.hdr[ki];
        const bool node_has = valid && (!(nh.flags & RF_DEF) || req_has(d, k, lane, nh, ws.words + CC.wsoff[ki]));
        uint64_t mask = 0;
        if (type == 0) {  // nextDomainTopologySpread: min count over the pod's domains, then the least-loaded node domain
            const uint64_t sup = ballot(kn && pod_has);
            int mn = wave_min_i32((kn && pod_has) ? cnt : INT32_MAX);
            if (info.w > 0 && __popcll(sup) < info.w) mn = 0;
            const int64_t c = (int64_t)cnt + self;
            const bool el = kn && node_has && c - (int64_t)mn <= (int64_t)info.z;
            const uint32_t key = el ? ((uint32_t)c << 8) | rk : 0xFFFFFFFFu;
            const uint32_t best = wave_min_u32(key);
            mask = best == 0xFFFFFFFFu ? 0ull : ballot(el && key == best);
        } else if (type == 2) {  // nextDomainAntiAffinity: empty domains allowed by pod and node
            mask = ballot(kn && cnt == 0 && pod_has && node_has);
        } else {  // nextDomainAffinity
            mask = ballot(kn && cnt > 0 && pod_has);
            if (!mask && self) {
                for (int pass = 0; pass < 2 && !mask; pass++) {
                    const bool c = kn && pod_has && (pass == 1 || node_has);
                    const uint32_t best = wave_min_u32(c ? rk : 0xFFFFFFFFu);
                    if (best != 0xFFFFFFFFu) mask = ballot(c && rk == best);
                }
            }
        }
        if (!mask) {
            ws.memo_ok = 0;
            return false;
        }
        int j = 0;
        while (j < nk && kidx[j] != ki) j++;
        if (j == nk) {
            kidx[nk] = ki;
            kmask[nk] = ~0ull;
            nk++;
        }
        kmask[j] &= mask;
    }
    // Compatible(r, topo) + Add: r[k] ∩ In[mask]
    bool fail = false, changed = false;
    for (int j = 0; j < nk; j++) {
        const int ki = kidx[j], k = CC.key[ki];
        if (lane == 0) {
            const ReqHdr A = ws.hdr[ki];
            uint64_t* aw = ws.words + CC.wsoff[ki];
            if (!(A.flags & RF_DEF)) {
                // undefined on the node: topo's In needs AllowUndefinedWellKnownLabels (an empty topo is DoesNotExist)
                if (kmask[j] != 0 && !(allow_wk && (CC.kflags[ki] & KF_WELL_KNOWN))) fail = true;
                ReqHdr o{};
                o.flags = RF_DEF;
                ws.hdr[ki] = o;
                aw[0] = kmask[j];
                changed = true;
            } else {
                ReqHdr B{};
                B.flags = RF_DEF;
                const uint64_t bw = kmask[j];
                ReqHdr O;
                uint64_t ow;
                const int cnt = req_intersect(d, k, A, aw, B, &bw, O, &ow);
                if (cnt == 0 && !op_notin_or_dne(req_op(A.flags, popc_words(aw, 1)))) fail = true;
                changed |= O.flags != A.flags || ow != aw[0];
                ws.hdr[ki] = O;
                aw[0] = ow;
            }
        }
    }
    fail = __builtin_amdgcn_readlane(fail ? 1 : 0, 0) != 0;  // lane 0's verdict, whole wave active here
    changed = __builtin_amdgcn_readlane(changed ? 1 : 0, 0) != 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (changed || fail) ws.memo_ok = 0;
    return !fail;
}

// Topology.Record for a committed placement (one wave).  The merged requirements are ws for the class's keys and the
// candidate's base digest (Ahdr / Aw) for the others; `host` is its hostname domain and `tmpl` its template (taints).
// Counts(pod): forward groups selecting the class, through the spread node filter (TopologyNodeFilter.Matches: the
// requirements are Compatible with one of the filter rows tg_frow — the owner's nodeSelector with each remaining
// required node-affinity term — with the AllowUndefinedWellKnownLabels option when allow_wk; the owner's
// tolerations); spread / affinity record a single-valued domain, anti-affinity and inverse groups record every value
// (requirement.Values(), the excluded set of a complement).
// The filter rows [r0, r0 + n) in one pass: lane i takes entry i of their concatenated key lists, and a row matches
// when none of its entries fails (n <= 64; kp_solve_prepare caps it).
__device__ inline bool topo_filter_compatible(const KpDev& d, const ClassCache& CC, const WaveScratch& ws,
                                              const ReqHdr* Ahdr, const uint64_t* Aw, int r0, int n, bool allow_wk,
                                              int lane, bool exnode = false) {
    const int i0 = d.cls_xkoff[r0], i1 = d.cls_xkoff[r0 + n];
    uint64_t bad = 0;  // rows with an incompatible key
    for (int i = i0 + lane; i - lane < i1; i += 64) {
        bool ok = true;
        int row = 0;
        if (i < i1) {
            while (d.cls_xkoff[r0 + row + 1] <= i) row++;
            const int rw = r0 + row;
            const int k = d.cls_xkeys[i];
            const ReqHdr B = d.cls_hdr[(size_t)rw * d.K + k];
            const uint64_t* bw = d.cls_words + (size_t)rw * d.DW + d.woff[k];
            const bool bno = op_notin_or_dne(req_op(B.flags, popc_words(bw, d.nw[k])));
            if (k == d.key_host && !exnode) {  // NodeClaim hostname In [placeholder]: only a complement without bounds admits it
                ok = (B.flags & RF_CMP) && !(B.flags & (RF_GT | RF_LT));
            } else {
                int ci = -1;
                for (int q = 0; q < CC.nck; q++)
                    if (CC.key[q] == k) ci = q;
                const ReqHdr A = ci >= 0 ? ws.hdr[ci] : Ahdr[k];
                const uint64_t* aw = ci >= 0 ? ws.words + CC.wsoff[ci] : Aw + d.woff[k];
                if (!(A.flags & RF_DEF)) ok = bno || (allow_wk && (d.kflags[k] & KF_WELL_KNOWN));
                else ok = !req_intersect_empty(d, k, A, aw, B, bw) || (bno && op_notin_or_dne(req_op(A.flags, popc_words(aw, d.nw[k]))));
            }
        }
        bad |= wave_or64(ok ? 0ull : 1ull << row);
    }
    return bad != (n >= 64 ? ~0ull : (1ull << n) - 1);
}

// exnode >= 0: the placement is on existing node exnode (its taints: ex_tol; its hostname is a real node name).
// born: the late identities created so far (the FFD kernel's; a probe's is *pt->born).
template <bool CT = false>
__device__ __forceinline__ void topo_record(const KpDev& d, const ClassCache& CC, const WaveScratch& ws, const ReqHdr* Ahdr,
                                         const uint64_t* Aw, int host, int tmpl, bool allow_wk, int lane, int exnode = -1,
                                         const ProbeTopo* pt = nullptr, uint64_t born = ~0ull) {
    if (CT && d.tg_late) born = *pt->born;
    for (int e = 0; e < CC.ntr; e++) {
        int g, ki;
        if (e < KP_CC_REC) {
            g = CC.tr[e];
            ki = CC.tr_ki[e];
        }
        else {  // beyond the cached entries: the class's list, and the group's key among the class keys
            g = d.cls_tr[d.cls_troff[CC.cls] + e];
            ki = -1;
            const int4 inf = d.tg_info[g];
            if (!(inf.x & TG_HOST))
                for (int i = 0; i < CC.nck; i++)
                    if (CC.key[i] == inf.y) ki = i;
        }
        if (d.tg_late) {  // a group Topology.Update has not created yet records nothing
            const int lt = d.tg_late[g];
            if (lt >= 0 && !((born >> lt) & 1ull)) continue;
        }
        const int4 info = d.tg_info[g];
        const int type = info.x & TG_TYPE;
        const bool inv = info.x & TG_INVERSE;
        if (!inv && type == 0) {  // TopologyNodeFilter.Matches
            const int pol = d.tg_pol[g], owner = d.tg_owner[g];
            const bool tolerated = exnode >= 0 ? ((d.ex_tol[(size_t)owner * d.EW + (exnode >> 6)] >> (exnode & 63)) & 1ull) != 0
                                               : ((d.tol[owner] >> tmpl) & 1ull) != 0;
            if ((pol & 2) && !tolerated) continue;
            if ((pol & 1) && owner != CC.cls) {
                const int2 fr = d.tg_frow[g];
                if (!topo_filter_compatible(d, CC, ws, Ahdr, Aw, fr.x, fr.y, allow_wk, lane, exnode >= 0)) continue;
            }
        }
        if (info.x & TG_HOST) {
            if (CT) {
                // a hostname-affinity group's domain becomes positive: one more domain holds a selected pod
                if (!inv && type == 1 && pt->ha[g] >= 0 && pt_hcnt(d, *pt, d.tg_hrow[g], host) == 0 && lane == 0)
                    pt->hpos[pt->ha[g]]++;
                pt_hadd(*pt, d.tg_hrow[g], host, lane);
            } else if (lane == 0) {
                const int old = atomicAdd(&d.tg_hcnt[(size_t)d.tg_hrow[g] * d.HN + host], 1);
                if (old == 0) atomicAdd(&d.tg_pos[g], 1);
            }
            continue;
        }
        const int k = info.y;
        const ReqHdr h = ki >= 0 ? ws.hdr[ki] : Ahdr[k];
        const uint64_t w = ki >= 0 ? ws.words[CC.wsoff[ki]] : ld_u64(Aw + d.woff[k]);
        if (!(h.flags & RF_DEF)) continue;  // Get() of an undefined key is Exists: no values
        if (!inv && type != 2 && ((h.flags & RF_CMP) || __popcll(w) != 1)) continue;
        if (CT) pt_row(d, *pt, g, lane);
        int32_t* cnt = CT ? pt->cnt : d.tg_cnt;
        uint64_t* known = CT ? pt->known : d.tg_known;
        if ((w >> lane) & 1ull) atomicAdd(&cnt[(size_t)g * 64 + lane], 1);
        if (lane == 0 && w) atomicOr((unsigned long long*)&known[g], (unsigned long long)w);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// ExistingNode.Add ([core] scheduling/existingnode.go) for a pod of a topology class on existing node j, one wave,
// after the caller found j tolerated, Compatible (XT) and with headroom: the requirement merge of the class's keys into
// the node's requirements (no undefined-label allowance), then Topology.AddRequirements with the node's own domains
// (hostname = the node's name: host row j).  On success ws holds the merged class keys.  nh_in / nw_in: the node's
// requirements digest when it is not d.ex_hdr's row j (a consolidation probe's copy of a node it changed).
template <bool CONS, bool CT = false>
__device__ inline bool existing_topo_try(const KpDev& d, const ClassCache& CC, WaveScratch& ws, int j, int lane,
                                         const ProbeTopo* pt = nullptr, const ReqHdr* nh_in = nullptr,
                                         const uint64_t* nw_in = nullptr) {
    const ReqHdr* nh = nh_in ? nh_in : d.ex_hdr + (size_t)j * d.K;
    const uint64_t* nwp = nw_in ? nw_in : d.ex_words + (size_t)j * d.DW;
    if (lane < CC.nck) {
        const int k = CC.key[lane], n = CC.nw[lane];
        const ReqHdr A = nh[k];
        const uint64_t* aw = nwp + CC.woff[lane];
        uint64_t* ow = ws.words + CC.wsoff[lane];
        ReqHdr O;
        if (((CC.kneutral >> lane) & 1u) || !(CC.hdr[lane].flags & RF_DEF)) {
            O = A;  // the class does not constrain the key: the node's requirement stands
            for (int i = 0; i < n; i++) ow[i] = (A.flags & RF_DEF) ? aw[i] : 0ull;
        } else if (!(A.flags & RF_DEF)) {
            O = CC.hdr[lane];  // undefined on the node: XT admitted it (NotIn / DoesNotExist)
            for (int i = 0; i < n; i++) ow[i] = CC.words[CC.wsoff[lane] + i];
        } else {
            req_intersect(d, k, A, aw, CC.hdr[lane], CC.words + CC.wsoff[lane], O, ow);
        }
        ws.hdr[lane] = O;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (CONS) return topo_narrow<CT>(d, CC, ws, j, false, lane, pt);
    return true;
}

// Commit of existing_topo_try: the node's requirements become the merged ones; when they changed, node j's XT column is
// recomputed for every class (as existing_merge does).
__device__ inline void existing_topo_commit(const KpDev& d, const ClassCache& CC, const WaveScratch& ws, int j, int lane) {
    ReqHdr* nh = d.ex_hdr + (size_t)j * d.K;
    uint64_t* nwp = d.ex_words + (size_t)j * d.DW;
    bool ch = false;
    if (lane < CC.nck) {
        const int k = CC.key[lane], n = CC.nw[lane];
        const ReqHdr O = ws.hdr[lane];
        const ReqHdr A = nh[k];
        ch = O.flags != A.flags || O.gt != A.gt || O.lt != A.lt || O.minv != A.minv;
        for (int i = 0; i < n; i++) {
            const uint64_t x = ws.words[CC.wsoff[lane] + i];
            const uint64_t y = (A.flags & RF_DEF) ? nwp[CC.woff[lane] + i] : 0ull;
            ch |= x != y;
            nwp[CC.woff[lane] + i] = x;
        }
        nh[k] = O;
    }
    if (!ballot(ch)) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // the merged requirements are visible to every lane
    const int w = j >> 6;
    const uint64_t bm = 1ull << (j & 63);
    for (int cc = lane; cc < d.C; cc += 64) {
        const bool ok = d.ex_static[j] && (d.ex_tol[(size_t)cc * d.EW + w] & bm) && node_compatible(d, nh, nwp, cc);
        if (ok) atomicOr((unsigned long long*)&d.XT[(size_t)cc * d.EW + w], (unsigned long long)bm);
        else atomicAnd((unsigned long long*)&d.XT[(size_t)cc * d.EW + w], (unsigned long long)~bm);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#define EV_STAMP(slot)                                                           \
    do {                                                                         \
        if (a.prof) {                                                            \
            const long long _t = __builtin_amdgcn_s_memtime();                   \
            if (lane == 0) atomicAdd((unsigned long long*)&a.prof[slot], (unsigned long long)(_t - _t0)); \
            _t0 = _t;                                                            \
        }                                                                        \
    } while (0)

// Wave-uniform result: does NodeClaim.Add(pod) succeed?  On success ws.opts / ws.hdr / ws.words hold the new state.
// TOPO: the class is constrained by topology groups (CF_TOPO_CONS): topo_narrow runs between the requirement merge
// and the type sweep, and keys carried only for narrowing (kneutral) merge as the base requirement.  RESV: the catalog
// has reserved offerings (offering compatibility over them, and the reservation step when E.resv_on).  The
// instantiations keep the topology and reservation code out of the common path.
// STRICT: ReservedOfferingModeStrict (provisioning); false: Fallback (disruption simulations never fail an Add for want
// of a reservation).  BE: the solve may run MIN_VALUES_POLICY=BestEffort (false compiles the relaxation bookkeeping out).
// TEAM: every wave of the block evaluates the same candidate (tb: this evaluation's TeamBuf, rank = wave, n waves):
// the requirement, topology and offering steps run in each wave alike, the type sweep is split over the waves by word,
// and one block barrier joins the partial sweeps; every wave ends with the same result in its ws.
template <bool TOPO, bool RESV = false, bool STRICT = true, bool BE = true, bool CT = false, bool TEAM = false>
__device__ __forceinline__ bool eval_wave(const KpDev& d, const EvalEnv& E, const ClassCache& CC, const EvalIn& a,
                                          WaveScratch& ws, int lane, TeamBuf* tb = nullptr, int trank = 0, int tn = 1,
                                          int* joins = nullptr) {
    const int TW = d.TW, T = d.T;
    long long _t0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    if (a.prof && lane == 0) atomicAdd((unsigned long long*)&a.prof[ST_EV_CALLS - ST_EV_REQ], 1ull);
    if (a.compat && !((CC.tol >> a.tmpl) & 1ull)) return false;
    const int nck = CC.nck;
    // request totals over the active axes (the first KP_LDS_AXES live in registers): the candidate's totals are read
    // past L1 here, so their latency overlaps the requirement merge
    int64_t tot[KP_LDS_AXES];
#pragma unroll
    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
        tot[ai] = 0;
        if (ai < d.n_active) {
            const int r = d.active_axes[ai];
            tot[ai] = (a.base_req ? ld_req(a.base_req + r) : 0) + (a.pod_req ? a.pod_req[r] : 0);
        }
    }

    // ---- requirements: Compatible + Add (lane = class key) ----
    bool fail = false, kill = false;
    uint64_t adm = ~0ull;
    int kmul = -1;
    bool rrow = false;  // this lane's key is the reservation-id label beyond 64 values (KF_RESV_ROWS)
    if (lane == 0) {
        ws.memo_ok = 1;
        if (BE) ws.n_minrel = 0;
    }
    // DoesNotExist-type elimination and the admissible value mask of a multi-valued key, from the merged requirement
    auto classify = [&](int k, const ReqHdr& O, const uint64_t* ow, int cnt) {
        const uint32_t kf = CC.kflags[lane];
        if (!(O.flags & RF_DEF)) return;
        if (kf & (KF_CAT_SINGLE | KF_CAT_MULTI | KF_RESV_ROWS)) kill = !op_notin_or_dne(req_op(O.flags, cnt));
        rrow = RESV && (kf & KF_RESV_ROWS) != 0;  // only catalogs with reserved offerings (the RESV instantiations)
        if (kf & KF_CAT_MULTI) {
            kmul = CC.kmulti[lane];
            const int nv = CC.nval[lane] < 64 ? CC.nval[lane] : 64;
            const uint64_t vm = nv >= 64 ? ~0ull : ((1ull << nv) - 1ull);
            if (!(O.flags & (RF_GT | RF_LT))) {  // Has(v) is the bit (complement: its absence)
                adm = ((O.flags & RF_CMP) ? ~ow[0] : ow[0]) & vm;
            } else {
                adm = 0;
                for (int v = 0; v < nv; v++)
                    if (req_has(d, k, v, O, ow)) adm |= 1ull << v;
            }
        }
    };
    if (lane < nck) {
        const int k = CC.key[lane];
        const int n = CC.nw[lane];
        const ReqHdr A = a.Ahdr[k];
        const uint64_t* aw = a.Aw + CC.woff[lane];
        const ReqHdr B = CC.hdr[lane];
        const uint64_t* bw = CC.words + CC.wsoff[lane];
        uint64_t* ow = ws.words + CC.wsoff[lane];
        ReqHdr O;
        int cnt;
        const int nb = CC.nbB[lane];
        if (TOPO && ((CC.kneutral >> lane) & 1u)) {
            // key present only for topology: the pod does not constrain it, the merge keeps the base requirement
            O = A;
            for (int i = 0; i < n; i++) ow[i] = (A.flags & RF_DEF) ? aw[i] : 0ull;
            cnt = 0;
        } else if (!(A.flags & RF_DEF)) {
            if (a.compat && !op_notin_or_dne(req_op(B.flags, nb)) && !(CC.kflags[lane] & KF_WELL_KNOWN)) fail = true;
            O = B;
            for (int i = 0; i < n; i++) ow[i] = bw[i];
            cnt = nb;
        } else {
            cnt = req_intersect(d, k, A, aw, B, bw, O, ow);
            if (a.compat && !(O.flags & RF_CMP) && cnt == 0) {
                const int na = popc_words(aw, n);
                if (!(op_notin_or_dne(req_op(B.flags, nb)) && op_notin_or_dne(req_op(A.flags, na)))) fail = true;
            }
        }
        ws.hdr[lane] = O;
        if (!TOPO) classify(k, O, ow, cnt);
    }
#define EV_REJ(slot) \
    do { \
        if (a.prof && lane == 0) atomicAdd((unsigned long long*)&a.prof[(slot) - ST_EV_REQ], 1ull); \
    } while (0)
    if (ballot(fail)) {
        EV_REJ(ST_REJ_REQ);
        return false;
    }
#ifdef KP_DIAG_SPLIT
    EV_STAMP(0);
#endif
    if (TOPO) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (!topo_narrow<CT>(d, CC, ws, a.host, a.compat, lane, E.pt, E.snap)) {
            EV_REJ(ST_REJ_TOPO);
            return false;
        }
        if (lane < nck) {
            const ReqHdr O = ws.hdr[lane];
            const uint64_t* ow = ws.words + CC.wsoff[lane];
            classify(CC.key[lane], O, ow, popc_words(ow, CC.nw[lane]));
        }
    }
#ifdef KP_DIAG_SPLIT
    EV_STAMP(1);
#else
    EV_STAMP(0);
#endif

    // ---- options ∧ V[class] ∧ ¬DoesNotExist-types of keys whose merged operator is In/Exists ----
    uint64_t myopt = 0;
    if (lane < TW) myopt = a.opts & CC.V[lane];
    uint64_t km = ballot(kill);
    while (km) {
        const int i = __ffsll((unsigned long long)km) - 1;
        km &= km - 1;
        if (lane < TW)
            myopt &= ~(lane < KP_DNE_TW ? CC.dne[i][lane]
                                        : (CC.kcat[i] >= 0 ? d.dne_mask[(size_t)CC.kcat[i] * TW + lane] : 0ull));
    }
    const uint64_t mm = ballot(kmul >= 0);
    const uint64_t mrr = RESV ? ballot(rrow) : 0ull;
    if (RESV && mrr) {
        // the reservation-id label beyond 64 values (rare; kept out of the type sweep below): a type's values are its
        // ResvTab rows' IDs (none: the label is DoesNotExist, left to the dne elimination above)
        const int i = __ffsll((unsigned long long)mrr) - 1;
        const ReqHdr O = ws.hdr[i];
        const uint64_t* ow = ws.words + CC.wsoff[i];
        for (int w = 0; w < TW; w++) {
            const uint64_t cw = rl64(myopt, w);
            if (cw == 0) continue;
            const int t = w * 64 + lane;
            bool ok = true;
            if ((cw >> lane) & 1ull) {
                const uint32_t tr = d.type_ro[t < T ? t : 0];
                const int r0 = (int)(tr >> 16) * 64 + (int)((tr >> 8) & 0xFFu), nr = (int)(tr & 0xFFu);
                ok = nr == 0;
                for (int r = 0; r < nr && !ok; r++) ok = req_has(d, CC.key[i], d.ro->ridv[r0 + r], O, ow);
            }
            const uint64_t m = ballot(ok);
            if (lane == w) myopt &= m;
        }
    }
    EV_STAMP(1);

    // ---- offerings over zone × capacity-type slots ----
    const bool need_off = a.force_off || (CC.flags & 1u);
    uint64_t mzc = ~0ull;
    if (need_off) {
        bool ok = false;
        if (lane < d.n_slots) {
            const int zid = E.slot_zoneid[lane];
            ok = role_adm(d, E, CC, ws, a.Ahdr, a.Aw, 0, E.slot_zone[lane]) &&
                 role_adm(d, E, CC, ws, a.Ahdr, a.Aw, 1, E.slot_ct[lane]) &&
                 (zid < 0 || role_adm(d, E, CC, ws, a.Ahdr, a.Aw, 2, zid)) &&
                 role_dneok(d, E, CC, ws, a.Ahdr, a.Aw, 3) && role_dneok(d, E, CC, ws, a.Ahdr, a.Aw, 4);
        }
        mzc = ballot(ok);
    }
    // reserved offerings: a type also has an offering when one of its reserved offerings is compatible (lane q: word q
    // of the compatible rows)
    const uint64_t mro =
        (RESV && E.ro && (need_off || E.resv_on)) ? resv_adm(d, E, CC, ws, a.Ahdr, a.Aw, lane) : 0ull;
    const bool mro_any = RESV && ballot(mro != 0) != 0;
    EV_STAMP(2);

    const int n_extra = d.n_active > KP_LDS_AXES ? d.n_active - KP_LDS_AXES : 0;
#ifdef KP_DIAG_SPLIT
    EV_STAMP(2);
#endif

    // ---- per type: Fits ∧ multi-valued labels ∧ offerings (64 types per ballot) ----
    WitnessAcc wit;
    wit.init(d, E, a.pod_req);
    uint64_t anyw = 0, newword = 0;
    for (int w = TEAM ? trank : 0; w < TW; w += TEAM ? tn : 1) {
        const uint64_t cw = rl64(myopt, w);
        if (cw == 0) continue;
        const int t = w * 64 + lane;
        bool keep = (cw >> lane) & 1ull;
        bool fit = true;
        int64_t av[KP_LDS_AXES];
        if (E.alloc) {
#pragma unroll
            for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                av[ai] = ai < d.lds_nstage ? E.alloc[ai * E.astride + t] : 0;
                fit &= !(tot[ai] > 0) | (tot[ai] <= av[ai]);
            }
        }
        for (int x = 0; x < n_extra; x++) {
            const int r = act_axis(d, KP_LDS_AXES + x);
            const int64_t tr = (a.base_req ? ld_req(a.base_req + r) : 0) + (a.pod_req ? a.pod_req[r] : 0);
            if (tr > 0) fit &= tr <= d.alloc[(size_t)r * T + (t < T ? t : 0)];
        }
        keep &= fit;
        uint64_t mmm = mm;
        while (mmm) {
            const int i = __ffsll((unsigned long long)mmm) - 1;
            mmm &= mmm - 1;
            const int m = rl32(kmul, i);
            const uint64_t am = rl64(adm, i);
            const uint64_t tm = E.multi16 ? (uint64_t)E.multi16[m * E.astride + t]
                                          : d.multi_mask[(size_t)m * T + (t < T ? t : 0)];
            keep &= (tm == 0) | ((tm & am) != 0);
        }
        if (need_off) {
            bool off = (E.avail[t] & mzc) != 0;
            if (RESV && mro_any) {  // the type's rows within their word
                const uint32_t tr = E.type_ro[t < T ? t : 0];
                off |= (shfl64(mro, (int)(tr >> 16)) & ro_span_bits(tr)) != 0;
            }
            keep &= off;
        }
        if (keep && wit.on) wit.add(av, tot, t);
        const uint64_t nb = ballot(keep);
        if (lane == w) newword = nb;
        anyw |= nb;
    }
#ifdef KP_DIAG_SPLIT
    EV_STAMP(3);
#endif
    if (TEAM) {
        // join the partial sweeps: every wave reads back all words, the OR and the team's witness arg-best
        if (wit.on) wit.reduce_wave();
        for (int w = trank; w < TW; w += tn)
            if (lane == w) tb->nw[w] = newword;
        if (lane == 0) {
            tb->any[trank] = anyw;
            tb->best[trank] = wit.best;
            tb->bt[trank] = wit.bt;
        }
        __syncthreads();
        (*joins)++;  // the caller's count of the joins reached (wave-uniform, a register once inlined)
        newword = lane < TW ? tb->nw[lane] : 0ull;
        anyw = 0;
        for (int r = 0; r < tn; r++) {
            anyw |= tb->any[r];
            wit.take(tb->best[r], tb->bt[r]);
        }
    }
#ifdef KP_DIAG_SPLIT
    EV_STAMP(4);
#else
    EV_STAMP(3);
#endif
    if (anyw == 0) {
        EV_REJ(ST_REJ_TYPES);
        return false;
    }

    // ---- minValues (Strict): distinct values per key over the remaining options ----
    if (a.tmpl >= 0 && ((E.min_tmpl_mask >> a.tmpl) & 1ull)) {
        const int* mk = d.min_keys + (size_t)a.tmpl * KP_MAX_CLASS_KEYS;
        for (int q = 0; q < KP_MAX_CLASS_KEYS; q++) {
            const int k = mk[q];
            if (k < 0) break;
            int ci = -1;
            for (int i = 0; i < nck; i++)
                if (CC.key[i] == k) ci = i;
            const ReqHdr h = ci >= 0 ? ws.hdr[ci] : a.Ahdr[k];
            if (!(h.flags & RF_MIN)) continue;
            int count = 0;
            const int kc = d.kcat[k];
            if (kc >= 0 && (d.kflags[k] & KF_CAT_MULTI)) {
                uint64_t acc = 0;
                for (int w = 0; w < TW; w++) {
                    const uint64_t nwd = rl64(newword, w);
                    const int t = w * 64 + lane;
                    if ((nwd >> lane) & 1ull) acc |= d.multi_mask[(size_t)d.kmulti[k] * T + t];
                }
                count = __popcll(wave_or64(acc));
            } else if (kc >= 0) {
                const int nwk = (d.nval[k] + 63) / 64;
                for (int i = lane; i < KP_MAX_MIN_WORDS; i += 64) ws.minbits[i] = 0;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                for (int w = 0; w < TW; w++) {
                    const uint64_t nwd = rl64(newword, w);
                    const int t = w * 64 + lane;
                    if ((nwd >> lane) & 1ull) {
                        const uint16_t v = d.type_val[(size_t)kc * T + t];
                        if (v < VAL_ABSENT && v < KP_MAX_MIN_WORDS * 64)
                            atomicOr((unsigned long long*)&ws.minbits[v >> 6], 1ull << (v & 63));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                int c = 0;
                for (int i = lane; i < nwk && i < KP_MAX_MIN_WORDS; i += 64) c += __popcll(ws.minbits[i]);
                for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
                count = c;
            }
            if (count < h.minv && !(BE && min_values_unmet(d, ws, k, count, lane))) {
                EV_REJ(ST_REJ_MIN);
                return false;
            }
        }
    }
    // ---- reservations (NodeClaim.Add's offeringsToReserve, ReservedOfferingModeStrict) ----
    // Every available reserved offering of a remaining type that the updated requirements are compatible with is
    // reserved for this NodeClaim: an ID it already holds, or one with capacity left.  The Add fails when a compatible
    // reserved offering exists but none can be reserved, or when the NodeClaim held reservations and none remain
    // (ReservedOfferingError).  Read-only here: the winner's commit takes / releases the capacity.  A rejection of
    // this kind needs every compatible ID the NodeClaim does not hold to be at capacity 0, and only a release can lift
    // a capacity from 0: such rejections stay memoised until commit_reservations reports one (FfdShared::rel_flag).
    bool rlive = false;
    if (RESV && E.resv_on) {
        const ResvTab& X = *E.ro;
        // the reservations the Add holds accumulate in ws.minbits (its minValues use is over)
        for (int i = lane; i < X.ridw; i += 64) ws.minbits[i] = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        bool cm = false, rm = false;
        for (int q = 0; q < X.w; q++) {  // 64 rows per step: row q * 64 + lane
            const int i = q * 64 + lane;
            const int tt = i < X.n ? X.type[i] : -1;
            const uint64_t wd = shfl64(newword, tt >= 0 ? tt >> 6 : 0);
            const bool comp = tt >= 0 && ((rl64(mro, q) >> lane) & 1ull) && ((wd >> (tt & 63)) & 1ull);
            const int rid = tt >= 0 ? X.rid[i] : 0;
            const uint64_t hw = shfl64(a.held, rid >> 6);
            const bool res = comp && (((hw >> (rid & 63)) & 1ull) || E.rcap[rid] > 0);
            cm |= ballot(comp) != 0;
            rm |= ballot(res) != 0;
            if (res) atomicOr((unsigned long long*)&ws.minbits[rid >> 6], 1ull << (rid & 63));
        }
        if (STRICT && ((cm && !rm) || (ballot(a.held != 0) && !rm))) return false;
        rlive = cm;
        if (lane == 0) ws.rlive = rlive ? 1 : 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane < TW) ws.opts[lane] = newword;
    // a NodeClaim that keeps reserved offerings is never quick-accepted (hr = -1): every Add recomputes its reservations
    wit.finish(d, E, tot, rlive || (a.tmpl >= 0 && ((E.min_tmpl_mask >> a.tmpl) & 1ull)), ws, lane, TEAM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    EV_STAMP(4);
    return true;
}

// The requirement merge of NodeClaim.Add(pod of class c) on the NodeClaim digest (Ahdr [K], Aw [DW]) is a no-op: for
// every key the class constrains (keys carried only for topology narrowing aside), the NodeClaim has the key and
// Requirement.Intersection leaves it as it is (header and values), and the pair passes Compatible.  Then the Add keeps
// the NodeClaim's requirements, so its options stay compatible and its offerings the same (one wave; ws.words is
// scratch).
__device__ inline bool merge_noop_at(const KpDev& d, WaveScratch& ws, const ReqHdr* Ahdr, const uint64_t* Aw, int c,
                                     int lane) {
    const int k0 = d.cls_koff[c], nck = d.cls_koff[c + 1] - k0;
    bool ok = true;
    if (lane < nck && !(d.cls_kneutral && d.cls_kneutral[k0 + lane])) {
        const int k = d.cls_keys[k0 + lane], n = d.nw[k];
        const ReqHdr A = Ahdr[k];
        const uint64_t* aw = Aw + d.woff[k];
        if (!(A.flags & RF_DEF)) {
            ok = false;  // the merge adds the key
        } else {
            const ReqHdr B = d.cls_hdr[(size_t)c * d.K + k];
            const uint64_t* bw = d.cls_words + (size_t)c * d.DW + d.woff[k];
            uint64_t* ow = ws.words + d.cls_wsoff[k0 + lane];
            ReqHdr O;
            const int cnt = req_intersect(d, k, A, aw, B, bw, O, ow);
            ok = O.flags == A.flags && O.gt == A.gt && O.lt == A.lt && O.minv == A.minv;
            for (int i = 0; i < n && ok; i++) ok = ow[i] == aw[i];
            if (!(O.flags & RF_CMP) && cnt == 0 &&
                !(op_notin_or_dne(req_op(B.flags, popc_words(bw, n))) && op_notin_or_dne(req_op(A.flags, popc_words(aw, n)))))
                ok = false;
        }
    }
    return ballot(!ok) == 0;
}

// merge_noop_at with the class's operands from the class cache (CC.cls is the class): keys, headers and words from LDS,
// so the NodeClaim's headers and words are the only global loads.
__device__ inline bool merge_noop_cc(const KpDev& d, const ClassCache& CC, WaveScratch& ws, const ReqHdr* Ahdr,
                                     const uint64_t* Aw, int lane) {
    bool ok = true;
    if (lane < CC.nck && !((CC.kneutral >> lane) & 1u)) {
        const int k = CC.key[lane], n = CC.nw[lane];
        const ReqHdr A = Ahdr[k];
        const uint64_t* aw = Aw + CC.woff[lane];
        if (!(A.flags & RF_DEF)) {
            ok = false;  // the merge adds the key
        } else {
            const ReqHdr B = CC.hdr[lane];
            const uint64_t* bw = CC.words + CC.wsoff[lane];
            uint64_t* ow = ws.words + CC.wsoff[lane];
            ReqHdr O;
            const int cnt = req_intersect(d, k, A, aw, B, bw, O, ow);
            ok = O.flags == A.flags && O.gt == A.gt && O.lt == A.lt && O.minv == A.minv;
            for (int i = 0; i < n && ok; i++) ok = ow[i] == aw[i];
            if (!(O.flags & RF_CMP) && cnt == 0 &&
                !(op_notin_or_dne(req_op(B.flags, popc_words(bw, n))) && op_notin_or_dne(req_op(A.flags, popc_words(aw, n)))))
                ok = false;
        }
    }
    return ballot(!ok) == 0;
}

// Write the merged class keys of a successful evaluation into NodeClaim slot n.
__device__ __forceinline__ void commit_reqs(const KpDev& d, const ClassCache& CC, const WaveScratch& ws, int n, int lane) {
    if (lane < CC.nck) {
        const int k = CC.key[lane];
        d.nc_hdr[(size_t)n * d.K + k] = ws.hdr[lane];
        for (int i = 0; i < CC.nw[lane]; i++) d.nc_words[(size_t)n * d.DW + CC.woff[lane] + i] = ws.words[CC.wsoff[lane] + i];
    }
}

// NodeClaim.Add for a NodeClaim that has already absorbed this pod class: Compatible/Add of the class requirements
// is idempotent (Intersection is idempotent and associative), and its label, DoesNotExist, multi-valued and
// offering filters are already applied to the options, which only shrink.  What remains is
// resources.Fits(requests + pod, Allocatable) over the options, then minValues.
template <bool BE = true>
__device__ __forceinline__ bool eval_fits_only(const KpDev& d, const EvalEnv& E, const EvalIn& a, WaveScratch& ws,
                                               int lane) {
    const int TW = d.TW, T = d.T;
    if (BE && lane == 0) ws.n_minrel = 0;
    int64_t tot[KP_LDS_AXES];
#pragma unroll
    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
        tot[ai] = 0;
        if (ai < d.n_active) {
            const int r = d.active_axes[ai];
            tot[ai] = ld_req(a.base_req + r) + a.pod_req[r];
        }
    }
    const int n_extra = d.n_active > KP_LDS_AXES ? d.n_active - KP_LDS_AXES : 0;
    WitnessAcc wit;
    wit.init(d, E, a.pod_req);
    uint64_t anyw = 0, newword = 0;
    for (int w = 0; w < TW; w++) {
        const uint64_t cw = rl64(a.opts, w);
        if (cw == 0) continue;
        const int t = w * 64 + lane;
        bool keep = (cw >> lane) & 1ull;
        int64_t av[KP_LDS_AXES];
#pragma unroll
        for (int ai = 0; ai < KP_LDS_AXES; ai++) {
            av[ai] = ai < d.lds_nstage ? E.alloc[ai * E.astride + t] : 0;
            keep &= !(tot[ai] > 0) | (tot[ai] <= av[ai]);
        }
        for (int x = 0; x < n_extra; x++) {
            const int r = act_axis(d, KP_LDS_AXES + x);
            const int64_t tr = ld_req(a.base_req + r) + a.pod_req[r];
            if (tr > 0) keep &= tr <= d.alloc[(size_t)r * T + (t < T ? t : 0)];
        }
        if (keep && wit.on) wit.add(av, tot, t);
        const uint64_t nb = ballot(keep);
        if (lane == w) newword = nb;
        anyw |= nb;
    }
    if (anyw == 0) return false;
    if ((E.min_tmpl_mask >> a.tmpl) & 1ull) {
        const int* mk = d.min_keys + (size_t)a.tmpl * KP_MAX_CLASS_KEYS;
        for (int q = 0; q < KP_MAX_CLASS_KEYS; q++) {
            const int k = mk[q];
            if (k < 0) break;
            const ReqHdr h = a.Ahdr[k];
            if (!(h.flags & RF_MIN)) continue;
            int count = 0;
            const int kc = d.kcat[k];
            if (kc >= 0 && (d.kflags[k] & KF_CAT_MULTI)) {
                uint64_t acc = 0;
                for (int w = 0; w < TW; w++) {
                    const uint64_t nwd = rl64(newword, w);
                    if ((nwd >> lane) & 1ull) acc |= d.multi_mask[(size_t)d.kmulti[k] * T + w * 64 + lane];
                }
                count = __popcll(wave_or64(acc));
            } else if (kc >= 0) {
                const int nwk = (d.nval[k] + 63) / 64;
                for (int i = lane; i < KP_MAX_MIN_WORDS; i += 64) ws.minbits[i] = 0;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                for (int w = 0; w < TW; w++) {
                    const uint64_t nwd = rl64(newword, w);
                    if ((nwd >> lane) & 1ull) {
                        const uint16_t v = d.type_val[(size_t)kc * T + w * 64 + lane];
                        if (v < VAL_ABSENT && v < KP_MAX_MIN_WORDS * 64)
                            atomicOr((unsigned long long*)&ws.minbits[v >> 6], 1ull << (v & 63));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                int c = 0;
                for (int i = lane; i < nwk && i < KP_MAX_MIN_WORDS; i += 64) c += __popcll(ws.minbits[i]);
                for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
                count = c;
            }
            if (count < h.minv && !(BE && min_values_unmet(d, ws, k, count, lane))) return false;
        }
    }
    if (lane < TW) ws.opts[lane] = newword;
    wit.finish(d, E, tot, (E.min_tmpl_mask >> a.tmpl) & 1ull, ws, lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    return true;
}

}  // namespace KP_WNS
using namespace KP_WNS;
