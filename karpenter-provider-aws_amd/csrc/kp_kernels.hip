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

#include "kp_device.h"
#include "kp_layout.h"

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
// NodeClaim.Add evaluation by one wave
// ------------------------------------------------------------------------------------------------
struct WaveScratch {
    ReqHdr hdr[KP_MAX_CLASS_KEYS];
    uint64_t words[KP_MAX_SCR_WORDS];
    uint64_t opts[KP_TW_MAX];
    uint64_t minbits[KP_MAX_MIN_WORDS];
};

struct EvalArgs {
    const ReqHdr* Ahdr;        // base requirements (NodeClaim, template or empty)
    const uint64_t* Aw;
    uint64_t opts;             // lane l < TW: InstanceTypeOptions word l
    const int64_t* base_req;   // [R] current requests (NodeClaim requests / daemon overhead) or null
    const int64_t* pod_req;    // [R] pod requests or null
    int cls;                   // class row (pod class, or C + j for template j)
    int tmpl;                  // template of the NodeClaim (taints, minValues keys)
    bool compat;               // apply taints + Requirements.Compatible (false for NewScheduler's template filter)
    bool force_off;            // always recheck offerings
};

// Merged requirement of key k: from the wave scratch if the class constrains k (index i >= 0), else base.
__device__ __forceinline__ bool adm_for(const KpDev& d, const EvalArgs& a, const WaveScratch& ws, int k, int i,
                                        int so, int v) {
    if (k < 0) return true;
    if (i >= 0) return req_has(d, k, v, ws.hdr[i], ws.words + so);
    const ReqHdr h = a.Ahdr[k];
    if (!(h.flags & RF_DEF)) return true;  // undefined + well-known offering key → AllowUndefined
    return req_has(d, k, v, h, a.Aw + d.woff[k]);
}
__device__ __forceinline__ bool dneok_for(const KpDev& d, const EvalArgs& a, const WaveScratch& ws, int k, int i,
                                          int so) {
    if (k < 0) return true;
    ReqHdr h;
    const uint64_t* w;
    if (i >= 0) {
        h = ws.hdr[i];
        w = ws.words + so;
    } else {
        h = a.Ahdr[k];
        if (!(h.flags & RF_DEF)) return true;
        w = a.Aw + d.woff[k];
    }
    return op_notin_or_dne(req_op(h.flags, popc_words(w, d.nw[k])));
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
    for (int o = 32; o >= 1; o >>= 1) x |= __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ int64_t wave_max64(int64_t x) {
    for (int o = 32; o >= 1; o >>= 1) {
        int64_t y = __shfl_xor(x, o);
        x = y > x ? y : x;
    }
    return x;
}

// Returns (wave-uniformly) whether NodeClaim.Add(pod) succeeds; on success ws.opts holds the remaining
// InstanceTypeOptions and ws.hdr/ws.words the merged requirements of the class's keys.
__device__ bool eval_wave(const KpDev& d, const EvalArgs& a, WaveScratch& ws, const int64_t* sAlloc,
                          const uint64_t* avail, int lane) {
    const int K = d.K, TW = d.TW, T = d.T;
    // Taints(template).ToleratesPod(pod)
    if (a.compat && !((d.tol[a.cls] >> a.tmpl) & 1u)) return false;
    const int k0 = d.cls_koff[a.cls];
    const int nck = d.cls_koff[a.cls + 1] - k0;

    // ---- Requirements: Compatible(nodeClaimReqs, podReqs, AllowUndefinedWellKnownLabels) + Add ----
    bool fail = false, kill = false;
    uint64_t adm = ~0ull;
    int kid = -1, kmul = -1, so = 0;
    if (lane < nck) {
        kid = d.cls_keys[k0 + lane];
        so = d.cls_wsoff[k0 + lane];
        const int n = d.nw[kid];
        const ReqHdr A = a.Ahdr[kid];
        const uint64_t* aw = a.Aw + d.woff[kid];
        const ReqHdr B = d.cls_hdr[(size_t)a.cls * K + kid];
        const uint64_t* bw = d.cls_words + (size_t)a.cls * d.DW + d.woff[kid];
        uint64_t* ow = ws.words + so;
        ReqHdr O;
        int cnt;
        const int nb = popc_words(bw, n);
        if (!(A.flags & RF_DEF)) {
            if (a.compat && !op_notin_or_dne(req_op(B.flags, nb)) && !(d.kflags[kid] & KF_WELL_KNOWN)) fail = true;
            O = B;
            for (int i = 0; i < n; i++) ow[i] = bw[i];
            cnt = nb;
        } else {
            cnt = req_intersect(d, kid, A, aw, B, bw, O, ow);
            if (a.compat && !(O.flags & RF_CMP) && cnt == 0) {
                const int na = popc_words(aw, n);
                if (!(op_notin_or_dne(req_op(B.flags, nb)) && op_notin_or_dne(req_op(A.flags, na)))) fail = true;
            }
        }
        ws.hdr[lane] = O;
        const uint32_t kf = d.kflags[kid];
        // types whose label is DoesNotExist survive only if the merged operator is NotIn / DoesNotExist
        if (kf & (KF_CAT_SINGLE | KF_CAT_MULTI)) kill = !op_notin_or_dne(req_op(O.flags, cnt));
        if (kf & KF_CAT_MULTI) {
            kmul = d.kmulti[kid];
            adm = 0;
            const int nv = d.nval[kid];
            for (int v = 0; v < nv && v < 64; v++)
                if (req_has(d, kid, v, O, ow)) adm |= 1ull << v;
        }
    }
    if (ballot(fail)) return false;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    // ---- candidate words: options ∧ V[class] ∧ ¬(DoesNotExist types of killed keys) ----
    uint64_t myopt = 0;
    if (lane < TW) myopt = a.opts & d.V[(size_t)a.cls * TW + lane];
    uint64_t km = ballot(kill);
    while (km) {
        const int i = __ffsll((unsigned long long)km) - 1;
        km &= km - 1;
        const int k = rl32(kid, i);
        if (lane < TW) myopt &= ~d.dne_mask[(size_t)d.kcat[k] * TW + lane];
    }
    const uint64_t mm = ballot(kmul >= 0);

    // ---- offerings: Available ∧ reqs.IsCompatible(offering.Requirements) over zone × capacity-type slots ----
    const bool need_off = a.force_off || (d.cls_flags[a.cls] & 1u);
    uint64_t mzc = ~0ull;
    if (need_off) {
        const uint64_t bz = ballot(lane < nck && kid == d.key_zone), bc = ballot(lane < nck && kid == d.key_ct),
                       bi = ballot(lane < nck && kid == d.key_zoneid), br = ballot(lane < nck && kid == d.key_resvid),
                       bt = ballot(lane < nck && kid == d.key_resvtype);
        const int iz = bz ? __ffsll((unsigned long long)bz) - 1 : -1, ic = bc ? __ffsll((unsigned long long)bc) - 1 : -1,
                  ii = bi ? __ffsll((unsigned long long)bi) - 1 : -1, ir = br ? __ffsll((unsigned long long)br) - 1 : -1,
                  it = bt ? __ffsll((unsigned long long)bt) - 1 : -1;
        const int sz = iz >= 0 ? rl32(so, iz) : 0, sc = ic >= 0 ? rl32(so, ic) : 0, si = ii >= 0 ? rl32(so, ii) : 0,
                  sr = ir >= 0 ? rl32(so, ir) : 0, st = it >= 0 ? rl32(so, it) : 0;
        bool ok = false;
        if (lane < d.n_slots) {
            ok = adm_for(d, a, ws, d.key_zone, iz, sz, d.slot_zone[lane]) &&
                 adm_for(d, a, ws, d.key_ct, ic, sc, d.slot_ct[lane]) &&
                 (d.slot_zoneid[lane] < 0 || adm_for(d, a, ws, d.key_zoneid, ii, si, d.slot_zoneid[lane])) &&
                 dneok_for(d, a, ws, d.key_resvid, ir, sr) && dneok_for(d, a, ws, d.key_resvtype, it, st);
        }
        mzc = ballot(ok);
    }

    // ---- per type: resources.Fits(requests, Allocatable) ∧ multi-valued labels ∧ offerings ----
    int64_t tot[KP_MAX_R];
#pragma unroll
    for (int ai = 0; ai < KP_MAX_R; ai++) {
        tot[ai] = 0;
        if (ai < d.n_active) {
            const int r = d.active_axes[ai];
            tot[ai] = (a.base_req ? a.base_req[r] : 0) + (a.pod_req ? a.pod_req[r] : 0);
        }
    }
    uint64_t anyw = 0, newword = 0;
    for (int w = 0; w < TW; w++) {
        const uint64_t cw = rl64(myopt, w);
        if (cw == 0) continue;
        const int t = w * 64 + lane;
        bool keep = (cw >> lane) & 1ull;
        if (keep) {
#pragma unroll
            for (int ai = 0; ai < KP_MAX_R; ai++) {
                if (ai < d.n_active && tot[ai] > 0) {
                    const int64_t av = (ai < KP_LDS_AXES) ? sAlloc[ai * KP_MAX_TYPES + t]
                                                          : d.alloc[(size_t)d.active_axes[ai] * T + t];
                    if (tot[ai] > av) keep = false;
                }
            }
            uint64_t mmm = mm;
            while (mmm) {
                const int i = __ffsll((unsigned long long)mmm) - 1;
                mmm &= mmm - 1;
                const int m = rl32(kmul, i);
                const uint64_t am = rl64(adm, i);
                const uint64_t tm = d.multi_mask[(size_t)m * T + t];
                if (tm && !(tm & am)) keep = false;
            }
            if (need_off && !(avail[t] & mzc)) keep = false;
        }
        const uint64_t nb = ballot(keep);
        if (lane == w) newword = nb;
        anyw |= nb;
    }
    if (anyw == 0) return false;

    // ---- minValues (MIN_VALUES_POLICY=Strict): SatisfiesMinValues over the remaining options ----
    if (a.tmpl >= 0) {
        const int* mk = d.min_keys + (size_t)a.tmpl * KP_MAX_CLASS_KEYS;
        for (int q = 0; q < KP_MAX_CLASS_KEYS; q++) {
            const int k = mk[q];
            if (k < 0) break;
            const uint64_t bk = ballot(lane < nck && kid == k);
            ReqHdr h;
            if (bk) h = ws.hdr[__ffsll((unsigned long long)bk) - 1];
            else h = a.Ahdr[k];
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
            if (count < h.minv) return false;
        }
    }
    if (lane < TW) ws.opts[lane] = newword;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    return true;
}

// ------------------------------------------------------------------------------------------------
// NodeClaimTemplate.InstanceTypeOptions
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void template_init_kernel(KpDev d) {
    __shared__ WaveScratch ws;
    const int j = blockIdx.x, lane = threadIdx.x;
    EvalArgs a;
    a.Ahdr = d.empty_hdr;
    a.Aw = d.empty_words;
    a.opts = lane < d.TW ? (d.tmpl_rows[(size_t)j * d.TW + lane] & d.nonneg[lane]) : 0;
    a.base_req = nullptr;
    a.pod_req = nullptr;
    a.cls = d.C + j;
    a.tmpl = j;
    a.compat = false;
    a.force_off = true;
    const bool ok = eval_wave(d, a, ws, nullptr, d.avail_zc, lane);
    if (lane < d.TW) d.tmpl_opts[(size_t)j * d.TW + lane] = ok ? ws.opts[lane] : 0;
    if (lane == 0) d.tmpl_ok[j] = ok ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// Solve: single-workgroup FFD
// ------------------------------------------------------------------------------------------------
struct FfdShared {
    int64_t sAlloc[KP_LDS_AXES * KP_MAX_TYPES];
    uint64_t sAvail[KP_MAX_TYPES];
    uint32_t key[KP_MAX_NC];   // len(Pods) by slice position
    uint32_t ncnt[KP_MAX_NC];  // len(Pods) by NodeClaim id
    uint16_t ord[KP_MAX_NC];   // s.newNodeClaims: NodeClaim id by slice position
    uint32_t rej[KP_MAX_NC / 32];
    WaveScratch ws[KP_NWAVES];
    uint64_t wmask[KP_NWAVES];
    int cand_pos[KP_NWAVES];
    int acc[KP_NWAVES];
    int sstack[64 * 5];
    int N, qhead, qcount, done, cur_pod, cur_cls, cur_shape, prev_shape;
    int dirty_kind, dirty_pos, seq, winner, n_cand, next_pos, scan_pos, err;
    long long st[ST_COUNT];
};

// ---- Go sort.Slice (pdqsort_func) over (key, ord) in LDS, one lane ----
struct LdsSlice {
    FfdShared& S;
    __device__ bool less(int i, int j) const { return S.key[i] < S.key[j]; }
    __device__ void swap(int i, int j) {
        uint32_t k = S.key[i];
        S.key[i] = S.key[j];
        S.key[j] = k;
        uint16_t o = S.ord[i];
        S.ord[i] = S.ord[j];
        S.ord[j] = o;
    }
};

__device__ __forceinline__ int go_bits_len(unsigned x) { return x ? 32 - __clz(x) : 0; }

__device__ void order2(const LdsSlice& d, int a, int b, int& swaps, int& x, int& y) {
    if (d.less(b, a)) {
        swaps++;
        x = b;
        y = a;
    } else {
        x = a;
        y = b;
    }
}
__device__ int median3(const LdsSlice& d, int a, int b, int c, int& swaps) {
    int x, y;
    order2(d, a, b, swaps, x, y);
    a = x;
    b = y;
    order2(d, b, c, swaps, x, y);
    b = x;
    c = y;
    order2(d, a, b, swaps, x, y);
    a = x;
    b = y;
    return b;
}
// choosePivot_func; hint: 0 unknown, 1 increasing, 2 decreasing
__device__ void choose_pivot(const LdsSlice& d, int a, int b, int& pivot, int& hint) {
    const int l = b - a;
    int swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
        if (l >= 50) {
            i = median3(d, i - 1, i, i + 1, swaps);
            j = median3(d, j - 1, j, j + 1, swaps);
            k = median3(d, k - 1, k, k + 1, swaps);
        }
        j = median3(d, i, j, k, swaps);
    }
    pivot = j;
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
}

__device__ void insertion_sort(LdsSlice& d, int a, int b) {
    for (int i = a + 1; i < b; i++)
        for (int j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
}
__device__ void sift_down(LdsSlice& d, int lo, int hi, int first) {
    int root = lo;
    for (;;) {
        int child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && d.less(first + child, first + child + 1)) child++;
        if (!d.less(first + root, first + child)) return;
        d.swap(first + root, first + child);
        root = child;
    }
}
__device__ void heap_sort(LdsSlice& d, int a, int b) {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(d, i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
        d.swap(first, first + i);
        sift_down(d, lo, i, first);
    }
}
__device__ int partition_go(LdsSlice& d, int a, int b, int pivot, bool& already) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && d.less(i, a)) i++;
    while (i <= j && !d.less(j, a)) j--;
    if (i > j) {
        d.swap(j, a);
        already = true;
        return j;
    }
    d.swap(i, j);
    i++;
    j--;
    for (;;) {
        while (i <= j && d.less(i, a)) i++;
        while (i <= j && !d.less(j, a)) j--;
        if (i > j) break;
        d.swap(i, j);
        i++;
        j--;
    }
    d.swap(j, a);
    already = false;
    return j;
}
__device__ int partition_equal(LdsSlice& d, int a, int b, int pivot) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
        while (i <= j && !d.less(a, i)) i++;
        while (i <= j && d.less(a, j)) j--;
        if (i > j) break;
        d.swap(i, j);
        i++;
        j--;
    }
    return i;
}
__device__ bool partial_insertion_sort(LdsSlice& d, int a, int b) {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
        while (i < b && !d.less(i, i - 1)) i++;
        if (i == b) return true;
        if (b - a < 50) return false;
        d.swap(i, i - 1);
        if (i - a >= 2) {
            for (int k = i - 1; k >= 1; k--) {
                if (!d.less(k, k - 1)) break;
                d.swap(k, k - 1);
            }
        }
        if (b - i >= 2) {
            for (int k = i + 1; k < b; k++) {
                if (!d.less(k, k - 1)) break;
                d.swap(k, k - 1);
            }
        }
    }
    return false;
}
__device__ void break_patterns(LdsSlice& d, int a, int b) {
    const int length = b - a;
    if (length >= 8) {
        uint64_t random = (uint64_t)length;
        const uint64_t modulus = 1ull << go_bits_len((unsigned)length);
        const int idx = a + (length / 4) * 2 - 1;
        for (int i = 0; i < 3; i++) {
            random ^= random << 13;
            random ^= random >> 7;
            random ^= random << 17;
            int other = (int)(random & (modulus - 1));
            if (other >= length) other -= length;
            d.swap(idx - 1 + i, a + other);
        }
    }
}
__device__ void reverse_range(LdsSlice& d, int a, int b) {
    int i = a, j = b - 1;
    while (i < j) {
        d.swap(i, j);
        i++;
        j--;
    }
}
// pdqsort_func with Go's recursion (smaller side first, then loop) on an explicit LDS stack.
__device__ void pdqsort_full(FfdShared& S, int n) {
    LdsSlice d{S};
    int* stk = S.sstack;
    int sp = 0;
    auto push = [&](int a, int b, int limit, int wb, int wp) {
        stk[sp * 5 + 0] = a;
        stk[sp * 5 + 1] = b;
        stk[sp * 5 + 2] = limit;
        stk[sp * 5 + 3] = wb;
        stk[sp * 5 + 4] = wp;
        sp++;
    };
    push(0, n, go_bits_len((unsigned)n), 1, 1);
    while (sp > 0) {
        sp--;
        int a = stk[sp * 5 + 0], b = stk[sp * 5 + 1], limit = stk[sp * 5 + 2];
        bool wasBalanced = stk[sp * 5 + 3], wasPartitioned = stk[sp * 5 + 4];
        for (;;) {
            const int length = b - a;
            if (length <= 12) {
                insertion_sort(d, a, b);
                break;
            }
            if (limit == 0) {
                heap_sort(d, a, b);
                break;
            }
            if (!wasBalanced) {
                break_patterns(d, a, b);
                limit--;
            }
            int pivot, hint;
            choose_pivot(d, a, b, pivot, hint);
            if (hint == 2) {
                reverse_range(d, a, b);
                pivot = (b - 1) - (pivot - a);
                hint = 1;
            }
            if (wasBalanced && wasPartitioned && hint == 1) {
                if (partial_insertion_sort(d, a, b)) break;
            }
            if (a > 0 && !d.less(a - 1, pivot)) {
                a = partition_equal(d, a, b, pivot);
                continue;
            }
            bool already = false;
            const int mid = partition_go(d, a, b, pivot, already);
            wasPartitioned = already;
            const int leftLen = mid - a, rightLen = b - mid;
            const int balanceThreshold = length / 8;
            if (leftLen < rightLen) {
                wasBalanced = leftLen >= balanceThreshold;
                push(mid + 1, b, limit, wasBalanced, wasPartitioned);  // continuation
                push(a, mid, limit, 1, 1);                             // recursive call first
            } else {
                wasBalanced = rightLen >= balanceThreshold;
                push(a, mid, limit, wasBalanced, wasPartitioned);
                push(mid + 1, b, limit, 1, 1);
            }
            break;
        }
    }
}

// first position in [s, n) whose key satisfies pred (wave 0, all lanes)
__device__ int wave_find_first_ge(const FfdShared& S, int s, int n, uint32_t v, int lane) {
    for (int base = s; base < n; base += 64) {
        const int p = base + lane;
        const uint64_t m = ballot(p < n && S.key[p] >= v);
        if (m) return base + __ffsll((unsigned long long)m) - 1;
    }
    return n;
}
__device__ int wave_find_first_gt(const FfdShared& S, int s, int n, uint32_t v, int lane) {
    for (int base = s; base < n; base += 64) {
        const int p = base + lane;
        const uint64_t m = ballot(p < n && S.key[p] > v);
        if (m) return base + __ffsll((unsigned long long)m) - 1;
    }
    return n;
}
// [a, e): element a moves to e-1, the rest shift left by one
__device__ void wave_rotate_left(FfdShared& S, int a, int e, int lane) {
    if (e - a < 2) return;
    const uint16_t fo = S.ord[a];
    const uint32_t fk = S.key[a];
    for (int base = a; base < e - 1; base += 64) {
        const int i = base + lane;
        uint16_t o = 0;
        uint32_t k = 0;
        if (i < e - 1) {
            o = S.ord[i + 1];
            k = S.key[i + 1];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (i < e - 1) {
            S.ord[i] = o;
            S.key[i] = k;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane == 0) {
        S.ord[e - 1] = fo;
        S.key[e - 1] = fk;
    }
}
// [q, n): element n-1 moves to q, the rest shift right by one
__device__ void wave_rotate_right(FfdShared& S, int q, int n, int lane) {
    if (n - q < 2) return;
    const uint16_t lo = S.ord[n - 1];
    const uint32_t lk = S.key[n - 1];
    for (int top = n - 1; top > q; top -= 64) {
        const int i = top - lane;
        uint16_t o = 0;
        uint32_t k = 0;
        if (i > q) {
            o = S.ord[i - 1];
            k = S.key[i - 1];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (i > q) {
            S.ord[i] = o;
            S.key[i] = k;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane == 0) {
        S.ord[q] = lo;
        S.key[q] = lk;
    }
}

// sort.Slice(s.newNodeClaims, by len(Pods)) given that the slice was sorted before exactly one change
// (dirty_kind 1: the NodeClaim at dirty_pos gained a pod; 2: a NodeClaim with 1 pod was appended).
// The stable move is exact whenever Go's pdqsort would resolve the change by insertionSort (n <= 12) or by
// partialInsertionSort (n >= 50 with an increasing pivot hint); every other case runs the full emulation.
__device__ void sort_emulate(FfdShared& S, int lane) {
    const int kind = S.dirty_kind, n = S.N;
    if (kind != 0 && n > 1) {
        const int dp = S.dirty_pos;
        bool inv;
        if (kind == 1) inv = (dp + 1 < n) && (S.key[dp + 1] < S.key[dp]);
        else inv = S.key[n - 2] > S.key[n - 1];
        if (inv) {
            bool fast = n <= 12;
            if (!fast) {
                LdsSlice d{S};
                int pivot, hint;
                choose_pivot(d, 0, n, pivot, hint);
                fast = (hint == 1 && n >= 50);
            }
            if (fast) {
                if (kind == 1) {
                    const int e = wave_find_first_ge(S, dp + 1, n, S.key[dp], lane);
                    wave_rotate_left(S, dp, e, lane);
                } else {
                    const int q = wave_find_first_gt(S, 0, n - 1, S.key[n - 1], lane);
                    wave_rotate_right(S, q, n, lane);
                }
                if (lane == 0) S.st[ST_SORT_FAST]++;
            } else {
                if (lane == 0) {
                    pdqsort_full(S, n);
                    S.st[ST_SORT_FULL]++;
                }
            }
        }
    }
    if (lane == 0) S.dirty_kind = 0;
}

// types whose Capacity exceeds a NodePool's remaining limits (filterByRemainingResources)
__device__ uint64_t limit_filter(const KpDev& d, int j, uint64_t o, int lane) {
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
                if (d.limit_set[(size_t)j * d.R + r] && d.cap[(size_t)r * d.T + t] > d.remaining[(size_t)j * d.R + r])
                    keep = false;
        }
        const uint64_t nb = ballot(keep);
        if (lane == w) out = nb;
    }
    return out;
}

// copy the merged class keys of a successful evaluation into NodeClaim slot n
__device__ void commit_reqs(const KpDev& d, const WaveScratch& ws, int cls, int n, int lane) {
    const int k0 = d.cls_koff[cls], nck = d.cls_koff[cls + 1] - k0;
    if (lane < nck) {
        const int k = d.cls_keys[k0 + lane], so = d.cls_wsoff[k0 + lane];
        d.nc_hdr[(size_t)n * d.K + k] = ws.hdr[lane];
        for (int i = 0; i < d.nw[k]; i++) d.nc_words[(size_t)n * d.DW + d.woff[k] + i] = ws.words[so + i];
    }
}

__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_kernel(KpDev d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    FfdShared& S = *reinterpret_cast<FfdShared*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = d.T, TW = d.TW, K = d.K, R = d.R, P = d.P;
    const int nstage = d.n_active < KP_LDS_AXES ? d.n_active : KP_LDS_AXES;
    for (int i = tid; i < nstage * KP_MAX_TYPES; i += blockDim.x) {
        const int ai = i / KP_MAX_TYPES, t = i % KP_MAX_TYPES;
        S.sAlloc[i] = t < T ? d.alloc[(size_t)d.active_axes[ai] * T + t] : 0;
    }
    for (int t = tid; t < KP_MAX_TYPES; t += blockDim.x) S.sAvail[t] = t < T ? d.avail_zc[t] : 0;
    for (int i = tid; i < KP_MAX_NC / 32; i += blockDim.x) S.rej[i] = 0;
    for (int p = tid; p < P; p += blockDim.x) {
        d.qbuf[p] = d.queue0[p];
        d.last_len[p] = 0;
        d.pod_result[p] = -1;
        d.pod_order[p] = -1;
    }
    if (tid == 0) {
        S.N = 0;
        S.qhead = 0;
        S.qcount = P;
        S.done = 0;
        S.prev_shape = -1;
        S.dirty_kind = 0;
        S.seq = 0;
        S.err = 0;
        for (int i = 0; i < ST_COUNT; i++) S.st[i] = 0;
    }
    __syncthreads();

    for (;;) {
        // ---- Queue.Pop ----
        if (tid == 0) {
            if (S.qcount == 0 || S.err) {
                S.done = 1;
            } else {
                const int p = d.qbuf[S.qhead];
                if (d.last_len[p] == S.qcount) {
                    S.done = 1;
                } else {
                    S.qhead = (S.qhead + 1 == P) ? 0 : S.qhead + 1;
                    S.qcount--;
                    S.cur_pod = p;
                    S.cur_cls = d.pod_cls[p];
                    S.cur_shape = d.pod_shape[p];
                    S.st[ST_POPPED]++;
                }
            }
        }
        __syncthreads();
        if (S.done) break;
        const int pod = S.cur_pod, cls = S.cur_cls;
        if (S.cur_shape != S.prev_shape)
            for (int i = tid; i < KP_MAX_NC / 32; i += blockDim.x) S.rej[i] = 0;
        // ---- sort.Slice(s.newNodeClaims, by len(Pods)) ----
        if (wave == 0) sort_emulate(S, lane);
        __syncthreads();
        if (tid == 0) {
            S.prev_shape = S.cur_shape;
            S.scan_pos = 0;
            S.winner = -1;
            S.st[ST_NC_SCANNED] += S.N;
        }
        __syncthreads();

        // ---- first in-flight NodeClaim (slice order) whose Add succeeds ----
        for (;;) {
            const int N = S.N, sp = S.scan_pos;
            if (sp >= N) break;
            const int p = sp + tid;
            bool c = false;
            if (p < N) {
                const int nc = S.ord[p];
                c = !((S.rej[nc >> 5] >> (nc & 31)) & 1u);
            }
            const uint64_t b = ballot(c);
            if (lane == 0) S.wmask[wave] = b;
            __syncthreads();
            if (tid == 0) {
                int n = 0;
                for (int w = 0; w < KP_NWAVES && n < KP_NWAVES; w++) {
                    uint64_t m = S.wmask[w];
                    while (m && n < KP_NWAVES) {
                        const int j = __ffsll((unsigned long long)m) - 1;
                        m &= m - 1;
                        S.cand_pos[n++] = sp + w * 64 + j;
                    }
                }
                S.n_cand = n;
                const int win_end = (sp + KP_NWAVES * 64 < N) ? sp + KP_NWAVES * 64 : N;
                S.next_pos = (n == KP_NWAVES) ? S.cand_pos[KP_NWAVES - 1] + 1 : win_end;
            }
            __syncthreads();
            if (wave < S.n_cand) {
                const int nc = S.ord[S.cand_pos[wave]];
                EvalArgs a;
                a.Ahdr = d.nc_hdr + (size_t)nc * K;
                a.Aw = d.nc_words + (size_t)nc * d.DW;
                a.opts = lane < TW ? d.nc_opts[(size_t)nc * TW + lane] : 0;
                a.base_req = d.nc_req + (size_t)nc * R;
                a.pod_req = d.pod_req + (size_t)pod * R;
                a.cls = cls;
                a.tmpl = d.nc_tmpl[nc];
                a.compat = true;
                a.force_off = false;
                const bool ok = eval_wave(d, a, S.ws[wave], S.sAlloc, S.sAvail, lane);
                if (lane == 0) {
                    S.acc[wave] = ok;
                    if (!ok) atomicOr(&S.rej[nc >> 5], 1u << (nc & 31));
                }
            }
            __syncthreads();
            if (tid == 0) {
                int win = -1;
                for (int w = 0; w < S.n_cand; w++)
                    if (S.acc[w]) {
                        win = w;
                        break;
                    }
                S.winner = win;
                S.st[ST_NC_EVALS] += S.n_cand;
                S.scan_pos = win >= 0 ? N : S.next_pos;
            }
            __syncthreads();
            if (S.winner >= 0) break;
        }

        if (S.winner >= 0) {
            const int w = S.winner;
            if (wave == w) {
                const int pos = S.cand_pos[w];
                const int nc = S.ord[pos];
                commit_reqs(d, S.ws[w], cls, nc, lane);
                if (lane < TW) d.nc_opts[(size_t)nc * TW + lane] = S.ws[w].opts[lane];
                for (int r = lane; r < R; r += 64) d.nc_req[(size_t)nc * R + r] += d.pod_req[(size_t)pod * R + r];
                if (lane == 0) {
                    S.ncnt[nc]++;
                    S.key[pos]++;
                    S.dirty_kind = 1;
                    S.dirty_pos = pos;
                    d.pod_result[pod] = nc;
                    d.pod_order[pod] = S.seq++;
                }
            }
        } else {
            // ---- new NodeClaim from the templates, in NodePool weight order ----
            for (int tb = 0; tb < d.NT; tb += KP_NWAVES) {
                const int j = tb + wave;
                if (j < d.NT) {
                    uint64_t o = (lane < TW && d.tmpl_ok[j]) ? d.tmpl_opts[(size_t)j * TW + lane] : 0;
                    o = limit_filter(d, j, o, lane);
                    bool ok = false;
                    if (ballot(o != 0)) {
                        EvalArgs a;
                        a.Ahdr = d.cls_hdr + (size_t)(d.C + j) * K;
                        a.Aw = d.cls_words + (size_t)(d.C + j) * d.DW;
                        a.opts = o;
                        a.base_req = d.daemon + (size_t)j * R;
                        a.pod_req = d.pod_req + (size_t)pod * R;
                        a.cls = cls;
                        a.tmpl = j;
                        a.compat = true;
                        a.force_off = false;
                        ok = eval_wave(d, a, S.ws[wave], S.sAlloc, S.sAvail, lane);
                    }
                    if (lane == 0) S.acc[wave] = ok;
                } else if (lane == 0) {
                    S.acc[wave] = 0;
                }
                __syncthreads();
                if (tid == 0) {
                    int win = -1;
                    for (int w = 0; w < KP_NWAVES && tb + w < d.NT; w++) {
                        S.st[ST_TMPL_EVALS]++;
                        if (S.acc[w]) {
                            win = w;
                            break;
                        }
                    }
                    S.winner = win;
                    if (win >= 0 && (S.N >= KP_MAX_NC || S.N >= d.NCcap)) {
                        S.err = 1;
                        S.winner = -1;
                    }
                }
                __syncthreads();
                if (S.winner >= 0) {
                    if (wave == S.winner) {
                        const int jj = tb + wave;
                        const int n = S.N;
                        // NewNodeClaim(template): requirements = template requirements, then the Add's merge
                        for (int k = lane; k < K; k += 64) d.nc_hdr[(size_t)n * K + k] = d.cls_hdr[(size_t)(d.C + jj) * K + k];
                        for (int i = lane; i < d.DW; i += 64)
                            d.nc_words[(size_t)n * d.DW + i] = d.cls_words[(size_t)(d.C + jj) * d.DW + i];
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        commit_reqs(d, S.ws[wave], cls, n, lane);
                        if (lane < TW) d.nc_opts[(size_t)n * TW + lane] = S.ws[wave].opts[lane];
                        for (int r = lane; r < R; r += 64)
                            d.nc_req[(size_t)n * R + r] = d.daemon[(size_t)jj * R + r] + d.pod_req[(size_t)pod * R + r];
                        // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
                        for (int r = 0; r < R; r++) {
                            if (!d.limit_set[(size_t)jj * R + r]) continue;
                            int64_t mx = INT64_MIN;
                            for (int w2 = 0; w2 < TW; w2++) {
                                const uint64_t ow = S.ws[wave].opts[w2];
                                if ((ow >> lane) & 1ull) {
                                    const int64_t c = d.cap[(size_t)r * T + w2 * 64 + lane];
                                    mx = c > mx ? c : mx;
                                }
                            }
                            mx = wave_max64(mx);
                            if (lane == 0) d.remaining[(size_t)jj * R + r] -= mx;
                        }
                        if (lane == 0) {
                            d.nc_tmpl[n] = jj;
                            S.ord[n] = (uint16_t)n;
                            S.key[n] = 1;
                            S.ncnt[n] = 1;
                            S.N = n + 1;
                            S.dirty_kind = 2;
                            S.dirty_pos = n;
                            d.pod_result[pod] = n;
                            d.pod_order[pod] = S.seq++;
                        }
                    }
                    break;
                }
            }
            // ---- Queue.Push(pod, relaxed=false) ----
            if (tid == 0 && S.winner < 0) {
                const int tail = (S.qhead + S.qcount) % P;
                d.qbuf[tail] = pod;
                S.qcount++;
                d.last_len[pod] = S.qcount;
            }
        }
        __syncthreads();
    }

    // ---- outputs ----
    const int N = S.N;
    for (int i = tid; i < N; i += blockDim.x) {
        d.nc_npods[i] = S.ncnt[i];
        d.nc_slice_pos[S.ord[i]] = i;
    }
    if (tid == 0) {
        d.nc_count[0] = N;
        d.err[0] = S.err;
        for (int i = 0; i < ST_COUNT; i++) d.stats[i] = S.st[i];
    }
}

// ------------------------------------------------------------------------------------------------
// FinalizeScheduling + Truncate(OrderByPrice, maxInstanceTypes) + SatisfiesMinValues
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void finalize_kernel(KpDev d) {
    __shared__ uint64_t s_key[KP_MAX_TYPES];
    __shared__ uint32_t s_rank[KP_MAX_TYPES];
    __shared__ uint16_t s_t[KP_MAX_TYPES];
    __shared__ uint64_t s_mzc;
    __shared__ int s_n;
    __shared__ uint64_t s_bits[KP_MAX_MIN_WORDS];
    __shared__ int s_ok;
    const int nc = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (nc >= d.nc_count[0]) return;
    const int T = d.T, TW = d.TW, M = d.M;
    const ReqHdr* H = d.nc_hdr + (size_t)nc * d.K;
    const uint64_t* W = d.nc_words + (size_t)nc * d.DW;
    if (tid == 0) {
        s_n = 0;
        s_ok = 1;
    }
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
    }
    __syncthreads();
    const uint64_t mzc = s_mzc;
    for (int t = tid; t < TW * 64; t += blockDim.x) {
        if (t >= T) continue;
        if (!((d.nc_opts[(size_t)nc * TW + (t >> 6)] >> (t & 63)) & 1ull)) continue;
        uint64_t m = d.avail_zc[t] & mzc;
        double price = 1.7976931348623157e308;  // math.MaxFloat64
        while (m) {
            const int s = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const double p = d.slot_price[(size_t)t * KP_MAX_SLOTS + s];
            price = p < price ? p : price;
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

hipError_t kp_launch_class_mask(const KpDev& d, hipStream_t s) {
    dim3 g(d.TW, d.C + d.NT);
    hipLaunchKernelGGL(class_mask_kernel, g, dim3(64), 0, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_template_init(const KpDev& d, hipStream_t s) {
    if (d.NT == 0) return hipSuccess;
    hipLaunchKernelGGL(template_init_kernel, dim3(d.NT), dim3(64), 0, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_ffd(const KpDev& d, hipStream_t s) {
    static bool attr = false;
    const size_t bytes = sizeof(FfdShared);
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)ffd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(ffd_kernel, dim3(1), dim3(KP_NWAVES * 64), bytes, s, d);
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
