// kp_kernels.hip — gfx950 kernels of the scheduling simulation (no MFMA: bitset / gather / compare work).
//
//   class_mask_kernel     pod-class × instance-type label compatibility sweep (V bitsets): one wave per
//                         (class, 64-type word), ballot over lanes.  Reference: compatible(it, reqs) =
//                         it.Requirements.Intersects(reqs) ([core] scheduling/nodeclaim.go
//                         filterInstanceTypesByRequirements; called at pkg/providers/instance/filter/filter.go:53).
//   template_init_kernel  NewScheduler's NodeClaimTemplate.InstanceTypeOptions =
//                         filterInstanceTypesByRequirements(instanceTypes[np], nct.Requirements, {}, {}, {}).
//   ffd_kernel            Scheduler.Solve: the whole first-fit-decreasing loop in ONE workgroup (8 waves), the
//                         queue, Go sort.Slice emulation, NodeClaim.Add for up to 8 candidate NodeClaims at once,
//                         new-NodeClaim creation from templates with NodePool limits.
//   finalize_kernel       FinalizeScheduling + InstanceTypes.Truncate(reqs, 60) (OrderByPrice, minValues),
//                         one workgroup per NodeClaim.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_ffd.h"


// ------------------------------------------------------------------------------------------------
// class × type label compatibility
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void class_mask_kernel(KpDev d) {
    const int w = blockIdx.x, c = blockIdx.y, lane = threadIdx.x;
    const int t = w * 64 + lane;
    bool bit = t < d.T;
    const int k0 = d.cls_koff[c], k1 = d.cls_koff[c + 1];
    for (int i = k0; i < k1 && bit; i++) {
        const int k = d.cls_keys[i];
        if (!(d.kflags[k] & KF_CAT_SINGLE)) continue;
        const uint16_t v = d.type_val[(size_t)d.kcat[k] * d.T + t];
        if (v >= VAL_ABSENT) continue;  // DoesNotExist types are handled by dne_mask at evaluation
        const ReqHdr h = d.cls_hdr[(size_t)c * d.K + k];
        bit = req_has(d, k, v, h, d.cls_words + (size_t)c * d.DW + d.woff[k]);
    }
    const uint64_t m = ballot(bit);
    if (lane == 0) d.V[(size_t)c * d.TW + w] = m;
}

// ------------------------------------------------------------------------------------------------
// existing nodes: working copies, headroom, static fit; then class × node Compatible ∧ tolerations (XT)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void existing_init_kernel(KpDev d) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.E) return;
    for (int k = 0; k < d.K; k++) d.ex_hdr[(size_t)j * d.K + k] = d.ex_hdr0[(size_t)j * d.K + k];
    for (int i = 0; i < d.DW; i++) d.ex_words[(size_t)j * d.DW + i] = d.ex_words0[(size_t)j * d.DW + i];
    // resources.Fits(requests + pod, available): any negative available fails; axes no pod requests are static
    bool ok = true;
    for (int r = 0; r < d.R; r++) {
        const int64_t av = d.ex_avail[(size_t)j * d.R + r], rq = d.ex_req[(size_t)j * d.R + r];
        bool act = false;
        for (int ai = 0; ai < d.n_active; ai++) act |= act_axis(d, ai) == r;
        if (av < 0 || (!act && rq > av)) ok = false;
    }
    d.ex_static[j] = ok ? 1 : 0;
    for (int ai = 0; ai < d.n_active; ai++) {
        const int r = act_axis(d, ai);
        d.ex_head[(size_t)ai * d.E + j] = d.ex_avail[(size_t)j * d.R + r] - d.ex_req[(size_t)j * d.R + r];
    }
}


__global__ __launch_bounds__(64) void existing_mask_kernel(KpDev d) {
    const int w = blockIdx.x, c = blockIdx.y, lane = threadIdx.x, j = w * 64 + lane;
    bool bit = j < d.E && d.ex_static[j] && ((d.ex_tol[(size_t)c * d.EW + w] >> lane) & 1ull);
    if (bit) bit = node_compatible(d, d.ex_hdr0 + (size_t)j * d.K, d.ex_words0 + (size_t)j * d.DW, c);
    const uint64_t m = ballot(bit);
    if (lane == 0) d.XT[(size_t)c * d.EW + w] = m;
}

// ------------------------------------------------------------------------------------------------
// NodeClaimTemplate.InstanceTypeOptions (NewScheduler): one wave per template
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void template_init_kernel(KpDev d) {
    __shared__ ClassCache CC;
    __shared__ WaveScratch ws;
    __shared__ Roles roles;
    const int j = blockIdx.x, lane = threadIdx.x;
    fill_class_cache(d, d.C + j, CC, lane, 64);
    if (lane < 5) {
        const int rk = lane == 0 ? d.key_zone : lane == 1 ? d.key_ct : lane == 2 ? d.key_zoneid : lane == 3 ? d.key_resvid : d.key_resvtype;
        roles.key[lane] = rk;
        roles.woff[lane] = rk >= 0 ? d.woff[rk] : 0;
        roles.nw[lane] = rk >= 0 ? d.nw[rk] : 0;
    }
    __syncthreads();
    EvalEnv E;
    E.pt = nullptr;
    E.snap = nullptr;
    E.alloc = nullptr;  // no requests: Fits({}, alloc) only needs non-negative allocatable (tmpl rows ∧ nonneg)
    E.astride = 0;
    E.avail = d.avail_zc;
    E.multi16 = nullptr;
    E.slot_zone = d.slot_zone;
    E.slot_ct = d.slot_ct;
    E.slot_zoneid = d.slot_zoneid;
    E.roles = &roles;
    E.min_tmpl_mask = d.min_keys[(size_t)j * KP_MAX_CLASS_KEYS] >= 0 ? (1ull << j) : 0ull;
    E.ro = d.ro;
    E.type_ro = d.type_ro;
    E.rcap = nullptr;
    E.resv_on = 0;  // NewScheduler's option filter: offerings only, no reservations
    EvalIn a;
    a.Ahdr = d.empty_hdr;
    a.Aw = d.empty_words;
    a.opts = lane < d.TW ? (d.tmpl_rows[(size_t)j * d.TW + lane] & d.nonneg[lane]) : 0;
    a.base_req = nullptr;
    a.pod_req = nullptr;
    a.tmpl = j;
    a.compat = false;
    a.force_off = true;
    a.prof = nullptr;
    a.host = 0;
    a.held = 0;
    const bool ok = d.ro ? eval_wave<false, true>(d, E, CC, a, ws, lane) : eval_wave<false>(d, E, CC, a, ws, lane);
    if (lane < d.TW) d.tmpl_opts[(size_t)j * d.TW + lane] = ok ? ws.opts[lane] : 0;
    if (lane == 0) d.tmpl_ok[j] = ok ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// Solve: the ffd_solve instantiations (kp_ffd.h), defined in kp_ffd_{base,resv,pref,pref_resv}.hip
// ------------------------------------------------------------------------------------------------
__global__ void ffd_kernel(KpDev d);
__global__ void ffd_topo_kernel(KpDev d);
__global__ void ffd_resv_kernel(KpDev d);
__global__ void ffd_resv_topo_kernel(KpDev d);
__global__ void ffd_pref_kernel(KpDev d);
__global__ void ffd_pref_topo_kernel(KpDev d);
__global__ void ffd_pref_resv_kernel(KpDev d);
__global__ void ffd_pref_resv_topo_kernel(KpDev d);
__global__ void ffd_hbm_kernel(KpDev d);
__global__ void ffd_topo_hbm_kernel(KpDev d);
__global__ void ffd_resv_hbm_kernel(KpDev d);
__global__ void ffd_resv_topo_hbm_kernel(KpDev d);
__global__ void ffd_pref_hbm_kernel(KpDev d);
__global__ void ffd_pref_topo_hbm_kernel(KpDev d);
__global__ void ffd_pref_resv_hbm_kernel(KpDev d);
__global__ void ffd_pref_resv_topo_hbm_kernel(KpDev d);


// ------------------------------------------------------------------------------------------------
// FinalizeScheduling + Truncate(OrderByPrice, maxInstanceTypes) + SatisfiesMinValues
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void finalize_kernel(KpDev d) {
    __shared__ uint64_t s_key[KP_MAX_TYPES];
    __shared__ uint32_t s_rank[KP_MAX_TYPES];
    __shared__ uint16_t s_t[KP_MAX_TYPES];
    __shared__ uint64_t s_mzc, s_mro[KP_RO_W];
    __shared__ int s_n;
    __shared__ uint64_t s_bits[KP_MAX_MIN_WORDS];
    __shared__ int s_ok;
    __shared__ int64_t s_tot[KP_MAX_R];
    const int nc = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (nc >= d.nc_count[0]) return;
    const int T = d.T, TW = d.TW, M = d.M;
    const ReqHdr* H = d.nc_hdr + (size_t)nc * d.K;
    const uint64_t* W = d.nc_words + (size_t)nc * d.DW;
    if (tid == 0) {
        s_n = 0;
        s_ok = 1;
        // FinalizeScheduling: a NodeClaim holding reservations gets ReservationIDLabel In [held IDs] (Requirements.Add:
        // the held IDs are admitted by the NodeClaim's requirement, so the intersection is In [held], minValues kept)
        bool any = false;
        for (int r = 0; d.resv_on && r < d.ro_ridw; r++) any |= d.nc_held[(size_t)nc * d.ro_ridw + r] != 0;
        if (any && d.key_resvid >= 0) {
            ReqHdr* hp = d.nc_hdr + (size_t)nc * d.K + d.key_resvid;
            uint64_t* wp = d.nc_words + (size_t)nc * d.DW + d.woff[d.key_resvid];
            ReqHdr o{};
            o.flags = RF_DEF | (hp->flags & RF_MIN);
            o.minv = hp->minv;
            *hp = o;
            for (int i = 0; i < d.nw[d.key_resvid]; i++) wp[i] = 0;
            for (int r = 0; r < d.ro_ridw; r++)
                for (uint64_t x = d.nc_held[(size_t)nc * d.ro_ridw + r]; x; x &= x - 1) {
                    const int v = d.ro->rid_vid[r * 64 + __ffsll((unsigned long long)x) - 1];
                    wp[v >> 6] |= 1ull << (v & 63);
                }
        }
    }
    __syncthreads();
    if (wave == 0) {
        // Offerings.Available().Compatible(reqs) over slots, reqs = NodeClaim requirements (hostname removed)
        bool ok = false;
        if (lane < d.n_slots) {
            auto adm = [&](int k, int v) -> bool {
                if (k < 0) return true;
                const ReqHdr h = H[k];
                if (!(h.flags & RF_DEF)) return true;
                return req_has(d, k, v, h, W + d.woff[k]);
            };
            auto dneok = [&](int k) -> bool {
                if (k < 0) return true;
                const ReqHdr h = H[k];
                if (!(h.flags & RF_DEF)) return true;
                return op_notin_or_dne(req_op(h.flags, popc_words(W + d.woff[k], d.nw[k])));
            };
            ok = adm(d.key_zone, d.slot_zone[lane]) && adm(d.key_ct, d.slot_ct[lane]) &&
                 (d.slot_zoneid[lane] < 0 || adm(d.key_zoneid, d.slot_zoneid[lane])) && dneok(d.key_resvid) &&
                 dneok(d.key_resvtype);
        }
        const uint64_t m = ballot(ok);
        if (lane == 0) s_mzc = m;
        // the reserved offerings, 64 rows per step (word q of s_mro)
        for (int q = 0; d.ro && q < d.ro_w; q++) {
            const int i = q * 64 + lane;
            bool rok = false;
            if (i < d.ro_n && d.ro->type[i] >= 0 && ((d.ro->avail[q] >> lane) & 1ull)) {
                auto adm = [&](int k, int v) -> bool {
                    if (k < 0) return true;
                    const ReqHdr h = H[k];
                    if (!(h.flags & RF_DEF)) return true;
                    return req_has(d, k, v, h, W + d.woff[k]);
                };
                const int zid = d.ro->zid[i], rt = d.ro->rtype[i];
                bool rtok;
                if (rt >= 0) {
                    rtok = adm(d.key_resvtype, rt);
                } else {
                    const ReqHdr h = d.key_resvtype >= 0 ? H[d.key_resvtype] : ReqHdr{};
                    rtok = !(h.flags & RF_DEF) ||
                           op_notin_or_dne(req_op(h.flags, popc_words(W + d.woff[d.key_resvtype], d.nw[d.key_resvtype])));
                }
                rok = adm(d.key_ct, d.ro->ctv) && adm(d.key_zone, d.ro->zone[i]) && (zid < 0 || adm(d.key_zoneid, zid)) &&
                      adm(d.key_resvid, d.ro->ridv[i]) && rtok;
            }
            const uint64_t rm = ballot(rok);
            if (lane == 0) s_mro[q] = rm;
        }
    }
    if (tid < d.R) s_tot[tid] = d.nc_req[(size_t)nc * d.R + tid];
    __syncthreads();
    const uint64_t mzc = s_mzc;
    for (int t = tid; t < TW * 64; t += blockDim.x) {
        if (t >= T) continue;
        if (!((d.nc_opts[(size_t)nc * TW + (t >> 6)] >> (t & 63)) & 1ull)) continue;
        // Fits(final requests, Allocatable): the quick-accept path applies Fits lazily (pick_witness)
        bool fit = true;
        for (int ai = 0; ai < d.n_active; ai++) {
            const int r = act_axis(d, ai);
            const int64_t tr = s_tot[r];
            if (tr > 0 && tr > d.alloc[(size_t)r * T + t]) fit = false;
        }
        if (!fit) continue;
        uint64_t m = d.avail_zc[t] & mzc;
        double price = 1.7976931348623157e308;  // math.MaxFloat64
        while (m) {
            const int s = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const double p = d.slot_price[(size_t)t * KP_MAX_SLOTS + s];
            price = p < price ? p : price;
        }
        if (d.ro) {  // the type's compatible available reserved offerings (its rows within their word)
            const uint32_t tr = d.type_ro[t];
            for (uint64_t rmk = tr ? s_mro[tr >> 16] & ro_span_bits(tr) : 0ull; rmk; rmk &= rmk - 1) {
                const double p = d.ro_price[(tr >> 16) * 64 + __ffsll((unsigned long long)rmk) - 1];
                price = p < price ? p : price;
            }
        }
        const int i = atomicAdd(&s_n, 1);
        s_key[i] = (uint64_t)__double_as_longlong(price);
        s_rank[i] = d.name_rank[t];
        s_t[i] = (uint16_t)t;
    }
    __syncthreads();
    const int n = s_n;
    for (int i = tid; i < n; i += blockDim.x) {
        const uint64_t ki = s_key[i];
        const uint32_t ri = s_rank[i];
        const uint16_t ti = s_t[i];
        int r = 0;
        for (int j = 0; j < n; j++) {
            const uint64_t kj = s_key[j];
            r += (kj < ki) || (kj == ki && (s_rank[j] < ri || (s_rank[j] == ri && s_t[j] < ti)));
        }
        if (r < M) d.nc_types[(size_t)nc * M + r] = ti;
    }
    if (tid == 0) {
        d.nc_nopts[nc] = n;
        d.nc_ntypes[nc] = n < M ? n : M;
    }
    __syncthreads();
    // Truncate: SatisfiesMinValues on the truncated list
    const int nt = n < M ? n : M;
    const int* mk = d.min_keys + (size_t)d.nc_tmpl[nc] * KP_MAX_CLASS_KEYS;
    for (int q = 0; q < KP_MAX_CLASS_KEYS; q++) {
        const int k = mk[q];
        if (k < 0) break;
        const ReqHdr h = H[k];
        if (!(h.flags & RF_MIN)) continue;
        for (int i = tid; i < KP_MAX_MIN_WORDS; i += blockDim.x) s_bits[i] = 0;
        __syncthreads();
        const int kc = d.kcat[k];
        for (int i = tid; i < nt; i += blockDim.x) {
            const int t = d.nc_types[(size_t)nc * M + i];
            if (kc < 0) continue;
            if (d.kflags[k] & KF_CAT_MULTI) {
                atomicOr((unsigned long long*)&s_bits[0], (unsigned long long)d.multi_mask[(size_t)d.kmulti[k] * T + t]);
            } else {
                const uint16_t v = d.type_val[(size_t)kc * T + t];
                if (v < VAL_ABSENT && v < KP_MAX_MIN_WORDS * 64)
                    atomicOr((unsigned long long*)&s_bits[v >> 6], 1ull << (v & 63));
            }
        }
        __syncthreads();
        if (tid == 0) {
            int c = 0;
            for (int i = 0; i < KP_MAX_MIN_WORDS; i++) c += __popcll(s_bits[i]);
            if (c < h.minv) s_ok = 0;
        }
        __syncthreads();
    }
    if (tid == 0) d.nc_valid[nc] = s_ok;
}

// ------------------------------------------------------------------------------------------------
// queue sort helpers (NewQueue: byCPUAndMemoryDescending, then creation time, then UID)
// ------------------------------------------------------------------------------------------------
__global__ void gather_key_kernel(const int64_t* __restrict__ field, int stride, int off, bool flip_desc,
                                  const int32_t* __restrict__ perm, uint64_t* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = perm[i];
    const int64_t v = field[(size_t)p * stride + off];
    uint64_t u = (uint64_t)v ^ 0x8000000000000000ull;  // order-preserving int64 → uint64
    if (flip_desc) u = ~u;
    out[i] = u;
}
__global__ void iota_kernel(int32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

// ------------------------------------------------------------------------------------------------
// launchers (called from kp_host.cpp)
// ------------------------------------------------------------------------------------------------
#include <hipcub/hipcub.hpp>

size_t kp_ffd_shared_bytes() { return sizeof(FfdShared); }
size_t kp_ffd_shared_bytes_topo();  // kp_ffd_base_topo.hip: FfdShared at KP_NWAVES_TOPO waves

// Lay out the FFD kernel's dynamic LDS for this solve (fills d.off_*, d.lds_*).  Returns false if even the
// quick-accept-free layout exceeds max_bytes.
static bool kp_ffd_plan_lds_tables(KpDev& d, int max_bytes);

// A solve is planned for KP_NC_FIRST in-flight NodeClaims with the allocatable table staged in LDS and the rest of LDS as
// quick-accept rows; a node-dense plan (NCcap above KP_NC_FIRST) reads the table from HBM and keeps as many slice entries
// in LDS as it holds (9 B per NodeClaim), or all of them in HBM.  Catalogs too large for the staged tables read the
// allocatable table, then the multi-valued label masks, from HBM.
bool kp_ffd_plan_lds(KpDev& d, int max_bytes) {
    d.alloc_global = d.NCcap > KP_NC_FIRST && d.alloc_act != nullptr;
    return kp_ffd_plan_lds_tables(d, max_bytes);
}

static bool kp_ffd_plan_lds_tables(KpDev& d, int max_bytes) {
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    // reserved offerings: the ResvTab header and the ReservationManager's capacities, then (small tables, up to
    // KP_RO_STAGE rows) the rows themselves (ffd_solve's staging)
    d.ro_stage = d.ro && d.ro_n <= KP_RO_STAGE ? 1 : 0;
    const size_t ro_bytes = !d.ro ? 0 : sizeof(ResvTab) + 4 * (size_t)((d.ro_nrid + 1) & ~1) +
                                        (d.ro_stage ? 24 * (size_t)((d.ro_n + 1) & ~1) + 8 * (size_t)d.ro_w : 0);
    // the topology instantiations run KP_NWAVES_TOPO waves: their fixed block is smaller
    size_t off = al(d.G > 0 ? kp_ffd_shared_bytes_topo() : sizeof(FfdShared));
    d.off_qw = (int)off;  // the queue window's pod requests, [64][R]
    off = al(off + 64 * 8 * (size_t)(d.R > 0 ? d.R : 1));
    int ncmax = d.NCcap < KP_MAX_NC ? d.NCcap : KP_MAX_NC;
    d.slice_hbm = 0;
    if (d.alloc_global) {
        const int tp0 = (d.T + 63) / 64 * 64;
        size_t fixed = off + 8 * (size_t)tp0 + (d.multi16 ? 2 * (size_t)d.n_multi * tp0 : 0) +
                       ro_bytes + (d.G > 0 ? sizeof(SnapRow) * (size_t)d.snap_rows : 0) + 256;
        const long room = ((long)max_bytes - (long)fixed) / 9;
        // more NodeClaims than LDS holds beside the fixed tables: the slice arrays go to HBM (the HBM instantiations)
        if (room < ncmax) d.slice_hbm = d.g_key != nullptr;
        if (room < ncmax && !d.slice_hbm) ncmax = room > 0 ? (int)room : 0;
    }
    d.lds_ncmax = ncmax;
    const size_t nsl = d.slice_hbm ? 0 : (size_t)ncmax;  // slice entries in LDS
    d.off_key = (int)off;
    off = al(off + 4 * nsl);
    d.off_ord = (int)off;
    off = al(off + 2 * nsl);
    d.off_last = (int)off;
    off = al(off + 2 * nsl);
    d.off_tmpl = (int)off;
    off = al(off + nsl);
    const int tp = (d.T + 63) / 64 * 64;
    d.lds_tpad = tp;
    d.lds_nstage = d.n_active < KP_LDS_AXES ? d.n_active : KP_LDS_AXES;
    d.off_alloc = (int)off;
    if (!d.alloc_global) off = al(off + 8 * (size_t)d.lds_nstage * tp);
    d.off_avail = (int)off;
    off = al(off + 8 * (size_t)tp);
    d.off_multi = (int)off;
    if (d.multi16) off = al(off + 2 * (size_t)d.n_multi * tp);
    d.off_ro = (int)off;
    if (d.ro) off = al(off + ro_bytes);
    d.off_tsnap = (int)off;
    if (d.G > 0) off = al(off + sizeof(SnapRow) * (size_t)d.snap_rows);
    d.off_hr = (int)off;
    if ((int)off > max_bytes) {
        // large catalogs: the staged allocatable, then the multi-valued label masks, are read from HBM instead
        if (!d.alloc_global && d.alloc_act) {
            d.alloc_global = 1;
            return kp_ffd_plan_lds_tables(d, max_bytes);
        }
        if (d.multi16) {
            d.multi16 = nullptr;
            return kp_ffd_plan_lds_tables(d, max_bytes);
        }
        return false;
    }
    d.lds_A = d.n_active <= KP_LDS_AXES ? d.n_active : 0;
    int nq = 0;
    if (d.lds_A > 0) {
        nq = (int)((max_bytes - (int)off) / (4 * d.lds_A));
        nq = nq < ncmax ? nq : ncmax;
    }
    d.lds_nq = nq;
    if (nq == 0) d.lds_A = 0;
    off += 4 * (size_t)d.lds_A * nq;
    d.lds_bytes = (int)off;
    return true;
}

hipError_t kp_launch_class_mask(const KpDev& d, hipStream_t s) {
    dim3 g(d.TW, d.C + d.NT);
    hipLaunchKernelGGL(class_mask_kernel, g, dim3(64), 0, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_existing(const KpDev& d, hipStream_t s) {
    if (d.E == 0) return hipSuccess;
    hipLaunchKernelGGL(existing_init_kernel, dim3((d.E + 255) / 256), dim3(256), 0, s, d);
    if (d.C > 0) hipLaunchKernelGGL(existing_mask_kernel, dim3(d.EW, d.C), dim3(64), 0, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_template_init(const KpDev& d, hipStream_t s) {
    if (d.NT == 0) return hipSuccess;
    hipLaunchKernelGGL(template_init_kernel, dim3(d.NT), dim3(64), 0, s, d);
    return hipGetLastError();
}
// Per-device kernel attributes: called by kp_ctx_create with the ctx's device current (every ctx, so a second ctx on
// another device of the same process gets them too; the call is idempotent and needs no process-wide flag).
hipError_t kp_ffd_set_attributes() {
    const void* ks[16] = {(const void*)ffd_kernel, (const void*)ffd_topo_kernel, (const void*)ffd_resv_kernel,
                          (const void*)ffd_resv_topo_kernel, (const void*)ffd_pref_kernel, (const void*)ffd_pref_topo_kernel,
                          (const void*)ffd_pref_resv_kernel, (const void*)ffd_pref_resv_topo_kernel,
                          (const void*)ffd_hbm_kernel, (const void*)ffd_topo_hbm_kernel, (const void*)ffd_resv_hbm_kernel,
                          (const void*)ffd_resv_topo_hbm_kernel, (const void*)ffd_pref_hbm_kernel,
                          (const void*)ffd_pref_topo_hbm_kernel, (const void*)ffd_pref_resv_hbm_kernel,
                          (const void*)ffd_pref_resv_topo_hbm_kernel};
    for (const void* k : ks) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, KP_LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t kp_launch_ffd(const KpDev& d, hipStream_t s) {
    const size_t bytes = (size_t)d.lds_bytes;
    // instantiation by solve features: reserved offerings (RESV), topology groups (TOPO), preference relaxation or
    // BestEffort minValues (PREF)
    const dim3 g(1), b((d.G > 0 ? KP_NWAVES_TOPO : KP_NWAVES) * 64);
    const bool pref = d.relax_next || d.best_effort;
    if (d.slice_hbm) {
        void (*k)(KpDev) = pref ? (d.ro ? (d.G > 0 ? ffd_pref_resv_topo_hbm_kernel : ffd_pref_resv_hbm_kernel)
                                        : (d.G > 0 ? ffd_pref_topo_hbm_kernel : ffd_pref_hbm_kernel))
                                : (d.ro ? (d.G > 0 ? ffd_resv_topo_hbm_kernel : ffd_resv_hbm_kernel)
                                        : (d.G > 0 ? ffd_topo_hbm_kernel : ffd_hbm_kernel));
        hipLaunchKernelGGL(k, g, b, bytes, s, d);
    } else if (pref) {
        if (d.ro && d.G > 0) hipLaunchKernelGGL(ffd_pref_resv_topo_kernel, g, b, bytes, s, d);
        else if (d.ro) hipLaunchKernelGGL(ffd_pref_resv_kernel, g, b, bytes, s, d);
        else if (d.G > 0) hipLaunchKernelGGL(ffd_pref_topo_kernel, g, b, bytes, s, d);
        else hipLaunchKernelGGL(ffd_pref_kernel, g, b, bytes, s, d);
    } else if (d.ro && d.G > 0) hipLaunchKernelGGL(ffd_resv_topo_kernel, g, b, bytes, s, d);
    else if (d.ro) hipLaunchKernelGGL(ffd_resv_kernel, g, b, bytes, s, d);
    else if (d.G > 0) hipLaunchKernelGGL(ffd_topo_kernel, g, b, bytes, s, d);
    else hipLaunchKernelGGL(ffd_kernel, g, b, bytes, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_finalize(const KpDev& d, int n_nodeclaims, hipStream_t s) {
    if (n_nodeclaims <= 0) return hipSuccess;
    hipLaunchKernelGGL(finalize_kernel, dim3(n_nodeclaims), dim3(256), 0, s, d);
    return hipGetLastError();
}

// Stable LSD radix passes: uid key asc, creation asc, memory desc, cpu desc  →  queue0 (pod indices).
// fields: [P][4] int64 {cpu, mem, creation, uidkey^sign}.  tmp buffers owned by the caller.
hipError_t kp_queue_sort(const int64_t* fields, int n, int32_t* perm_a, int32_t* perm_b, uint64_t* keys_a,
                         uint64_t* keys_b, void* temp, size_t* temp_bytes, hipStream_t s, int32_t** result) {
    if (temp == nullptr) {
        size_t b = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b, keys_a, keys_b, perm_a, perm_b, n, 0, 64, s);
        *temp_bytes = b;
        return e;
    }
    const int bs = 256, gs = (n + bs - 1) / bs;
    hipLaunchKernelGGL(iota_kernel, dim3(gs), dim3(bs), 0, s, perm_a, n);
    const int order[4] = {3, 2, 1, 0};
    const bool desc[4] = {false, false, true, true};
    int32_t* pin = perm_a;
    int32_t* pout = perm_b;
    for (int pass = 0; pass < 4; pass++) {
        hipLaunchKernelGGL(gather_key_kernel, dim3(gs), dim3(bs), 0, s, fields, 4, order[pass], desc[pass], pin, keys_a, n);
        size_t b = *temp_bytes;
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, b, keys_a, keys_b, pin, pout, n, 0, 64, s);
        if (e != hipSuccess) return e;
        int32_t* x = pin;
        pin = pout;
        pout = x;
    }
    *result = pin;
    return hipGetLastError();
}
