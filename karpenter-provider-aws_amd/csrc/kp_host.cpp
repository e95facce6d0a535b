// kp_host.cpp — C-ABI implementation of libkpsim.so (include/kpsim.h): dictionary encoding of the catalog
// and of a solve's requirements into device digests, device buffer management, kernel orchestration and
// result decoding.  All scheduling decisions are made by the gfx950 kernels in kp_kernels.hip; this file
// only encodes inputs and decodes outputs (there is no host fallback: without a device every call fails
// with KP_E_DEVICE).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kpsim.h"
#include "kp_gosort_host.h"
#include "kp_cons.h"
#include "kp_launch.h"
#include "kp_layout.h"

size_t kp_ffd_shared_bytes();
size_t kp_ffd_shared_bytes_topo();
bool kp_ffd_plan_lds(KpDev& d, int max_bytes);
hipError_t kp_launch_class_mask(const KpDev& d, hipStream_t s);
hipError_t kp_launch_template_init(const KpDev& d, hipStream_t s);
hipError_t kp_launch_existing(const KpDev& d, hipStream_t s);
hipError_t kp_launch_ffd(const KpDev& d, hipStream_t s);
hipError_t kp_ffd_set_attributes();
hipError_t kp_cons_set_attributes();
hipError_t kp_launch_finalize(const KpDev& d, int n_nodeclaims, hipStream_t s);
bool kp_cons_plan_lds(const KpDev& d, KpCons& k, int max_bytes);
hipError_t kp_launch_select_kernel(const KpLaunch& g, hipStream_t s);
hipError_t kp_launch_consolidate(const KpDev& d, const KpCons& k, int n_workers, hipStream_t s, KpDev* d_dev,
                                 KpCons* d_k);
hipError_t kp_launch_cons_chunk_max(const KpDev& d, int64_t* cmax0, hipStream_t s);
hipError_t kp_launch_multi_union(const KpCons& k, int nu, uint64_t* ubits, int32_t* rcand, int2* ulist, int32_t* ulen,
                                 const int32_t* queue0, hipStream_t s);
hipError_t kp_launch_cons_prep(const int32_t* queue0, int P, int32_t* rank, const int32_t* pending, int n_pending,
                               uint64_t* pend_bits, hipStream_t s);
hipError_t kp_queue_sort(const int64_t* fields, int n, int32_t* perm_a, int32_t* perm_b, uint64_t* keys_a,
                         uint64_t* keys_b, void* temp, size_t* temp_bytes, hipStream_t s, int32_t** result);

namespace {

using clk = std::chrono::steady_clock;
double ns_since(clk::time_point t0) { return std::chrono::duration<double, std::nano>(clk::now() - t0).count(); }

// ---------------------------------------------------------------------------------------------
// label dictionaries
// ---------------------------------------------------------------------------------------------
bool go_atoi(const char* s, int64_t& out) {  // strconv.Atoi (64-bit)
    size_t n = strlen(s), i = 0;
    bool neg = false;
    if (n == 0) return false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
    }
    if (i >= n) return false;
    unsigned __int128 v = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (unsigned)(s[i] - '0');
        if (v > (unsigned __int128)1 << 63) return false;
    }
    if (!neg && v > (unsigned __int128)INT64_MAX) return false;
    out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
    return true;
}

const char* const kWellKnown[] = {
    // karpv1.WellKnownLabels ([core] pkg/apis/v1/labels.go)
    "karpenter.sh/nodepool", "topology.kubernetes.io/zone", "topology.kubernetes.io/region",
    "node.kubernetes.io/instance-type", "kubernetes.io/arch", "kubernetes.io/os", "karpenter.sh/capacity-type",
    "node.kubernetes.io/windows-build",
    // AWS additions, pkg/apis/v1/labels.go:31-57
    "karpenter.k8s.aws/capacity-reservation-id", "karpenter.k8s.aws/capacity-reservation-type",
    "karpenter.k8s.aws/instance-hypervisor", "karpenter.k8s.aws/instance-encryption-in-transit-supported",
    "karpenter.k8s.aws/instance-category", "karpenter.k8s.aws/instance-capacity-flex", "karpenter.k8s.aws/instance-family",
    "karpenter.k8s.aws/instance-generation", "karpenter.k8s.aws/instance-size", "karpenter.k8s.aws/instance-local-nvme",
    "karpenter.k8s.aws/instance-cpu", "karpenter.k8s.aws/instance-cpu-manufacturer",
    "karpenter.k8s.aws/instance-cpu-sustained-clock-speed-mhz", "karpenter.k8s.aws/instance-memory",
    "karpenter.k8s.aws/instance-ebs-bandwidth", "karpenter.k8s.aws/instance-network-bandwidth",
    "karpenter.k8s.aws/instance-gpu-name", "karpenter.k8s.aws/instance-gpu-manufacturer",
    "karpenter.k8s.aws/instance-gpu-count", "karpenter.k8s.aws/instance-gpu-memory",
    "karpenter.k8s.aws/instance-accelerator-name", "karpenter.k8s.aws/instance-accelerator-manufacturer",
    "karpenter.k8s.aws/instance-accelerator-count", "topology.k8s.aws/zone-id",
};
bool well_known(const std::string& k) {
    for (auto* w : kWellKnown)
        if (k == w) return true;
    return false;
}
// karpv1.NormalizedLabels + topology.ebs.csi.aws.com/zone (pkg/operator/operator.go:71)
// normalize without a std::string temporary (launch-request encoding)
const char* normalize_c(const char* k) {
    static const std::pair<const char*, const char*> m[] = {
        {"failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone"},
        {"failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region"},
        {"beta.kubernetes.io/arch", "kubernetes.io/arch"},
        {"beta.kubernetes.io/os", "kubernetes.io/os"},
        {"beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type"},
        {"topology.ebs.csi.aws.com/zone", "topology.kubernetes.io/zone"},
    };
    for (auto& p : m)
        if (!strcmp(k, p.first)) return p.second;
    return k;
}
std::string normalize(const char* k) {
    static const std::pair<const char*, const char*> m[] = {
        {"failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone"},
        {"failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region"},
        {"beta.kubernetes.io/arch", "kubernetes.io/arch"},
        {"beta.kubernetes.io/os", "kubernetes.io/os"},
        {"beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type"},
        {"topology.ebs.csi.aws.com/zone", "topology.kubernetes.io/zone"},
    };
    for (auto& p : m)
        if (!strcmp(k, p.first)) return p.second;
    return k;
}

struct KeyDict {
    std::string name;
    std::unordered_map<std::string, int> ids;
    std::vector<std::string> vals;
    int id(const std::string& v) {
        auto it = ids.find(v);
        if (it != ids.end()) return it->second;
        int i = (int)vals.size();
        ids.emplace(v, i);
        vals.push_back(v);
        slots.clear();  // the fast index no longer covers every value: find_fast falls back to find
        return i;
    }
    int find(const std::string& v) const {
        auto it = ids.find(v);
        return it == ids.end() ? -1 : it->second;
    }
    // open-addressing FNV-1a index over vals for C-string lookups without std::string temporaries (launch-request
    // encoding); rebuilt by freeze() after the dictionary stops growing (catalog upload)
    std::vector<int32_t> slots;
    static uint64_t hash(const char* s) {
        uint64_t h = 1469598103934665603ull;
        for (; *s; s++) h = (h ^ (uint8_t)*s) * 1099511628211ull;
        return h;
    }
    void freeze() {
        size_t cap = 16;
        while (cap < vals.size() * 2) cap <<= 1;
        slots.assign(cap, -1);
        for (int i = 0; i < (int)vals.size(); i++) {
            size_t h = hash(vals[i].c_str()) & (cap - 1);
            while (slots[h] >= 0) h = (h + 1) & (cap - 1);
            slots[h] = i;
        }
    }
    int find_fast(const char* v) const {
        if (slots.empty()) return find(v);
        const size_t mask = slots.size() - 1;
        for (size_t h = hash(v) & mask;; h = (h + 1) & mask) {
            const int i = slots[h];
            if (i < 0) return -1;
            if (!strcmp(vals[i].c_str(), v)) return i;
        }
    }
};

struct Dicts {
    std::vector<KeyDict> keys;
    std::unordered_map<std::string, int> kid;
    int key(const std::string& k) {
        auto it = kid.find(k);
        if (it != kid.end()) return it->second;
        int i = (int)keys.size();
        kid.emplace(k, i);
        keys.emplace_back();
        keys.back().name = k;
        return i;
    }
    int find_key(const std::string& k) const {
        auto it = kid.find(k);
        return it == kid.end() ? -1 : it->second;
    }
    // FNV index over the key names for C-string lookups (launch-request encoding); rebuilt by freeze_keys()
    std::vector<int32_t> kslots;
    void freeze_keys() {
        size_t cap = 16;
        while (cap < keys.size() * 2) cap <<= 1;
        kslots.assign(cap, -1);
        for (int i = 0; i < (int)keys.size(); i++) {
            size_t h = KeyDict::hash(keys[i].name.c_str()) & (cap - 1);
            while (kslots[h] >= 0) h = (h + 1) & (cap - 1);
            kslots[h] = i;
        }
    }
    int find_key_fast(const char* k) const {
        if (kslots.empty() || kslots.size() < keys.size() * 2) return find_key(k);
        const size_t mask = kslots.size() - 1;
        for (size_t h = KeyDict::hash(k) & mask;; h = (h + 1) & mask) {
            const int i = kslots[h];
            if (i < 0) return -1;
            if (!strcmp(keys[i].name.c_str(), k)) return i;
        }
    }
};

// host requirement (value ids) used while encoding digests
struct HReq {
    int key = -1;
    bool complement = false;
    std::vector<int> vals;  // sorted unique
    bool has_gt = false, has_lt = false;
    int64_t gt = 0, lt = 0;
    bool has_min = false;
    int minv = 0;
};

template <class T>
struct DBuf {  // device buffer, grow-only; freed by its destructor (the owning ctx sets the device first)
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    hipError_t ensure(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
        size_t c = count ? count : 1;
        hipError_t e = hipMalloc((void**)&p, c * sizeof(T));
        if (e == hipSuccess) n = c;
        return e;
    }
    hipError_t upload(const std::vector<T>& v, hipStream_t s) {
        hipError_t e = ensure(v.size());
        if (e != hipSuccess || v.empty()) return e;
        return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
    }
    hipError_t upload(const T* v, size_t count, hipStream_t s) {
        hipError_t e = ensure(count);
        if (e != hipSuccess || count == 0) return e;
        return hipMemcpyAsync(p, v, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
    }
};

struct PrefExpansion {
    std::vector<kp_pod_class> classes;
    std::vector<int32_t> relax_next;  // per expanded class; empty when no class can relax
    kp_solve_input in{};
    // storage of the stage classes' arrays (pointers are set once every stage exists)
    std::vector<std::vector<kp_requirement>> reqs;
    std::vector<std::vector<kp_toleration>> tols;
    std::vector<std::vector<kp_topology_term>> terms;
    // per expanded class: the spread node filter (MakeTopologyNodeFilter: the nodeSelector with each remaining required
    // node-affinity term, ORed; no preference) and, when a preferred node-affinity term is in force, the strict
    // requirements (NewStrictPodRequirements: nodeSelector + the first remaining required term) that give podDomains
    std::vector<std::vector<std::vector<kp_requirement>>> filt;
    std::vector<std::vector<kp_requirement>> strict;
    std::vector<uint8_t> has_strict;
    std::vector<int32_t> origin;  // per expanded class: its input class
    int n_input = 0;
};

// Persistent worker threads of a ctx for the host-side batch work of kp_launch_select (request encoding, result
// expansion): run(k, fn) calls fn(0..k-1) across the workers and the calling thread and returns when all are done.
class WorkerPool {
  public:
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size() + 1; }
    void grow(int n) {  // at most n - 1 workers (the caller is the n-th)
        while ((int)th_.size() < n - 1) th_.emplace_back([this] { loop(); });
    }
    // false when a task threw (the exception is contained in its worker: one escaping a std::thread would
    // std::terminate the caller's process); the caller reports it as a KP_E_* status
    bool run(int k, const std::function<void(int)>& fn) {
        if (k <= 1 || th_.empty()) {
            try {
                for (int i = 0; i < k; i++) fn(i);
            } catch (...) {
                return false;
            }
            return true;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            next_ = 0;
            tasks_ = k;
            left_ = k;
            failed_ = false;
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return left_ == 0; });
        fn_ = nullptr;
        return !failed_;
    }

  private:
    void work() {
        for (;;) {
            int i;
            const std::function<void(int)>* f;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!fn_ || next_ >= tasks_) return;
                i = next_++;
                f = fn_;
            }
            bool ok = true;
            try {
                (*f)(i);
            } catch (...) {
                ok = false;
            }
            std::lock_guard<std::mutex> g(mu_);
            if (!ok) failed_ = true;
            if (--left_ == 0) done_.notify_all();
        }
    }
    void loop() {
        int seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int next_ = 0, tasks_ = 0, left_ = 0, gen_ = 0;
    bool stop_ = false, failed_ = false;
};

// Pinned host staging buffer, grow-only (launch-request tables: DMA without the pageable-copy staging).
template <class T>
struct PinBuf {
    T* p = nullptr;
    size_t n = 0;
    PinBuf() = default;
    PinBuf(const PinBuf&) = delete;
    PinBuf& operator=(const PinBuf&) = delete;
    ~PinBuf() {
        if (p) hipHostFree(p);
    }
    hipError_t ensure(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr;
        n = 0;
        const size_t c = count ? count : 1;
        hipError_t e = hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = c;
        return e;
    }
};

}  // namespace

// ---------------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------------
struct kp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t lstream2 = nullptr;          // kp_launch_select: odd sub-batches (their kernels overlap the even ones' tails)
    // kp_device_opts.devices[1..n): one ctx per further device (own stream, own copies of the catalog and of the
    // prepared consolidation pass).  Catalog uploads / patches and kp_consolidate_prepare run on every device (one host
    // thread each); kp_consolidate_execute splits the probe range into one contiguous shard per device and gathers the
    // shards' results into the caller's buffer (≤ 40 B per probe, an in-process host gather).
    std::vector<kp_ctx*> peers;
    std::string err;
    int pref_policy = KP_PREFERENCE_RESPECT;  // kp_device_opts solver parameters
    int reserved_capacity = 1;
    // catalog (host copies)
    bool have_catalog = false;
    uint64_t epoch = 0;
    int T = 0, TW = 0, R = 0, Kcat = 0, n_multi = 0, n_slots = 0;
    std::vector<std::string> resource_names, type_names;
    Dicts cat;                               // catalog dictionaries (keys 0..Kcat-1 are catalog label keys)
    std::vector<uint32_t> cat_kflags;        // per catalog key: KF_CAT_SINGLE / KF_CAT_MULTI
    std::vector<int> cat_multi;              // per catalog key: multi index or -1
    std::vector<int64_t> cap_rt, alloc_rt;   // [R][T]
    std::vector<uint64_t> avail_zc;          // [T]
    std::vector<int> off_type, off_slot;     // per offering row
    std::vector<double> slot_price;          // [T][KP_MAX_SLOTS]
    std::vector<int32_t> slot_zone, slot_ct, slot_zoneid;
    std::vector<uint64_t> h_multi_mask;      // [n_multi][T] value masks of the multi-valued keys (topology domains)
    std::vector<uint8_t> h_multi_state;      // [n_multi][T] KP_LABEL_* of those keys
    int key_zone = -1, key_ct = -1, key_zoneid = -1, key_resvid = -1, key_resvtype = -1;
    // catalog device tables
    DBuf<uint16_t> d_type_val, d_multi16;
    bool multi16_ok = false;
    DBuf<uint64_t> d_multi_mask, d_dne_mask, d_avail_zc, d_nonneg;
    DBuf<int64_t> d_alloc, d_cap;
    DBuf<double> d_slot_price;
    DBuf<int32_t> d_slot_zone, d_slot_ct, d_slot_zoneid;
    DBuf<uint32_t> d_name_rank;
    // solve
    bool prepared = false, executed = false;
    Dicts sol;                               // per-solve dictionaries = catalog ∪ requirement strings
    KpDev dev{};
    int P = 0, C = 0, NT = 0, K = 0, DW = 0;
    std::vector<int> tmpl_np;                // template → input nodepool index
    std::vector<int64_t> h_remaining;        // NodePool limits at solve start (re-applied by every execute)
    DBuf<uint32_t> d_kflags, d_cls_flags;
    DBuf<uint64_t> d_tol;
    DBuf<ReqHdr> d_ex_hdr0, d_ex_hdr;
    DBuf<uint64_t> d_ex_words0, d_ex_words, d_ex_tol, d_XT;
    DBuf<int64_t> d_ex_avail, d_ex_req, d_ex_head;
    DBuf<uint8_t> d_ex_static;
    DBuf<int32_t> d_cls_xkoff, d_cls_xkeys;
    DBuf<int32_t> d_kcat, d_kmulti, d_woff, d_nw, d_nval, d_vbase, d_cls_koff, d_cls_keys, d_cls_wsoff, d_min_keys;
    DBuf<uint8_t> d_val_isint, d_limit_set;
    DBuf<int64_t> d_val_int, d_daemon, d_remaining, d_pod_req, d_sort_fields, d_nc_req, d_stats;
    DBuf<uint64_t> d_tmpl_lmask;             // [NT][TW] FFD kernel: types within each template's remaining limits
    DBuf<ReqHdr> d_cls_hdr, d_nc_hdr, d_empty_hdr;
    DBuf<uint64_t> d_cls_words, d_V, d_tmpl_rows, d_tmpl_opts, d_nc_words, d_nc_opts, d_empty_words, d_keys_a, d_keys_b;
    DBuf<int32_t> d_tmpl_ok, d_pod_cls, d_pod_shape, d_perm_a, d_perm_b, d_nc_tmpl, d_qbuf, d_last_len, d_pod_result,
        d_pod_order, d_nc_count, d_nc_npods, d_nc_slice_pos, d_nc_nopts, d_nc_valid, d_nc_types, d_nc_ntypes, d_err;
    DBuf<char> d_sort_temp;
    size_t sort_temp_bytes = 0;
    double ns_prep = 0, ns_exec = 0, ns_fin = 0;
    hipEvent_t ev[6] = {};
    double kernel_ms[5] = {};
    int64_t cycles[37] = {};  // FFD phases (s_memtime): pop, sort, scan+eval, templates, commit, full pdqsort
    bool any_min_values = false;             // some template requirement carries minValues
    bool min_multi = false;                  // ... on a multi-valued catalog key (zone, capacity type, ...)
    std::vector<uint8_t> cons_mutcls;        // per (expanded) class: its NotIn/DoesNotExist merge can change a node's
                                             // requirements in a way a later decision sees (MUT probes)
    // consolidation probes
    DBuf<int32_t> d_retry, d_rank, d_cand_i, d_cand_off, d_cand_pods, d_pending, d_ring, d_ring_last, d_next, d_pnode;
    DBuf<double> d_cand_price;
    DBuf<int64_t> d_cand_cap, d_delta, d_alloc_act, d_cons_stats, d_cmax0, d_alloc_stage;
    // kp_solve_prepare's per-pod host arrays, kept across calls
    std::vector<int32_t> h_uid_p;
    std::vector<uint64_t> h_uid_k;
    std::vector<int32_t> h_shape_tab;
    int nc_cap_once = 0;                     // > 0: the next prepare plans for this many NodeClaims (after an overflow)
    int last_plan_nc = 0;                    // in-flight NodeClaim capacity of the last prepare
    bool nc_overflow = false;                // the last fetch found the solve out of in-flight NodeClaim capacity
    DBuf<uint64_t> d_pend_bits, d_pbits;
    DBuf<uint64_t> d_ubits;                  // multi-node probes' union list (multi_union_kernel): queue-position bits,
    DBuf<int32_t> d_rcand, d_ulen;           // candidate by queue position, list length
    DBuf<int2> d_ulist;                      // entries
    DBuf<uint64_t> d_init;
    DBuf<kp_probe_result> d_probe_out;
    DBuf<int32_t> d_rec_i;                   // kp_consolidate_command's read-back of the chosen REPLACE probe
    DBuf<int64_t> d_prof_probe;              // KPSIM_PROFILE: per-probe cycles
    DBuf<ReqHdr> d_rec_hdr;
    DBuf<uint64_t> d_rec_words;
    // MUT probes: per-probe flags (single-node by candidate, multi-node by prefix) and the per-worker node requirement
    // copies of the MUT variant
    DBuf<int32_t> d_mut_s, d_mut_m, d_ov_slot;
    DBuf<ReqHdr> d_ov_hdr;
    DBuf<uint64_t> d_ov_words;
    int cons_n_mut = 0;                      // probes of the prepared pass that run on the MUT variant
    // kp_consolidate_command reuses the last full pass and the last read-back of the prepared pass (a command right
    // after kp_consolidate_execute, or a retry after KP_E_BUFFER, launches nothing); cons_gen moves whenever device
    // tables or the prepared pass change, which makes both stale
    uint64_t cons_gen = 0;
    uint64_t pass_gen = ~0ull;
    int pass_mode = -1;
    std::vector<kp_probe_result> pass_rows;  // probes of the last full pass of pass_mode
    uint64_t rec_gen = ~0ull;
    int rec_mode = -1, rec_probe = -1;
    kp_probe_result rec_row{};
    int32_t rec_ri[4 + 64 + 1] = {};
    std::vector<ReqHdr> rec_h;
    std::vector<uint64_t> rec_w;
    int64_t n_pass_launches = 0, n_readbacks = 0;  // since the last kp_consolidate_prepare (kp_consolidate_stats)
    KpCons cons{};                         // prepared consolidation pass (device pointers set per execute)
    bool cons_prepared = false;
    // device prep of the prepared cluster (queue sort, ranks, pending bits, class / template / existing-node masks)
    // is reused by later kp_consolidate_execute calls until any entry point that rewrites device tables runs
    bool cons_prep_valid = false;
    int32_t* cons_q0 = nullptr;
    int cons_max_candidates = 100, cons_n_pending = 0;
    std::vector<int32_t> cons_off;           // candidate pod CSR offsets
    double cons_ms[3] = {};                  // device prep (sort, masks), probe kernel, whole call
    int64_t cons_stats[CS_COUNT] = {};
    // launch selection (kp_launch_select): raw offering rows, incl. reserved offerings
    bool has_reserved = false, launch_ok = true;
    std::string solve_unsupported;           // catalog the Solve tables cannot hold (launch selection still works)
    // reserved offerings in Solve (ReservationManager): <= 64 per catalog
    bool ro_ok = true;
    std::string ro_why;  // why the reserved offerings do not fit ResvTab (Solve / consolidation refuse with it)
    bool wide_resvid = false;                // the reservation-id label has > 64 values (no type value masks for it)
    bool resvid_rows = false;                // ... and every type's label is its ResvTab rows' IDs (KF_RESV_ROWS)
    // reserved offerings (ResvTab rows, kp_layout.h; padding rows have type -1 and offering -1)
    std::vector<int32_t> ro_type, ro_zone, ro_zid, ro_rid, ro_ridv, ro_rtype;
    std::vector<int32_t> ro_rid_vid;         // [nrid] reservation-id value id of each reservation
    std::vector<uint64_t> ro_avail;          // [w]
    std::vector<int32_t> ro_off;             // offering row of reserved-offering row i
    std::vector<uint32_t> type_ro;           // [T] packed span of the type's rows
    std::vector<int32_t> rcap0;              // [nrid]
    std::vector<double> ro_price;            // [rows]
    ResvTab h_ro{};                          // header with the device pointers below
    std::vector<ResvTab> h_ro_up;            // upload staging of h_ro (outlives the async copy)
    DBuf<ResvTab> d_ro;
    DBuf<int32_t> d_ro_type, d_ro_zone, d_ro_zid, d_ro_rid, d_ro_ridv, d_ro_rtype, d_ro_rid_vid;
    DBuf<uint64_t> d_ro_avail;
    DBuf<uint32_t> d_type_ro;
    DBuf<uint64_t> d_nc_held;
    DBuf<int32_t> d_rcap0, d_nc_rlive;
    DBuf<double> d_ro_price;
    DBuf<int32_t> d_trace;                   // KPSIM_TRACE_POD diagnostics
    std::string launch_err;
    std::vector<std::vector<std::pair<int, int>>> type_single;  // [T] (catalog key, value id) with Len() == 1
    int ct_vid[3] = {-1, -1, -1};            // value ids of on-demand / spot / reserved in the capacity-type dictionary
    std::vector<int32_t> l_off_begin, l_off_val, l_ct, l_rt, l_rcap;
    std::vector<double> l_price;
    std::vector<uint8_t> l_avail, l_exotic;
    DBuf<int32_t> d_l_off_begin, d_l_off_val, d_l_ct, d_l_rt, d_l_rcap, d_l_hdr, d_l_types;
    DBuf<uint64_t> d_l_over;
    DBuf<double> d_l_price;
    DBuf<uint8_t> d_l_avail, d_l_exotic;
    DBuf<KlReq> d_l_req;
    DBuf<KlKey> d_l_keys[2];                 // two staging sets: sub-batch b uses set b & 1 (kp_launch_select)
    DBuf<KlMinKey> d_l_mins[2];
    DBuf<uint64_t> d_l_words[2];
    DBuf<int64_t> d_l_rq;
    PinBuf<KlReq> p_l_req;                   // pinned staging of the launch tables and results
    PinBuf<int64_t> p_l_rq;
    PinBuf<KlKey> p_l_keys[2];
    PinBuf<KlMinKey> p_l_mins[2];
    PinBuf<uint64_t> p_l_words[2], p_l_over;
    PinBuf<int32_t> p_l_hdr, p_l_types;
    PinBuf<int32_t> p_pcls, p_pshape;        // kp_solve_prepare's per-pod arrays (pinned: DMA uploads)
    PinBuf<int64_t> p_preq, p_fields;
    WorkerPool pool;                         // host threads of kp_launch_select's batch work
    double launch_ms[6] = {};                // Σ launch kernel, whole call; host phases: encode, merge + upload,
                                             // waits for the downloads, result expansion
    int launch_nsub = 0;                     // sub-batches of the last call
    double launch_busy_ms = 0;               // union of the call's kernel intervals (overlapping sub-batch kernels)
    hipEvent_t lev[3 * KL_MAX_SUB] = {};     // per sub-batch: kernel start, kernel end, download landed
    // topology (kp_solve_prepare encodes the groups; execute resets the counts from the *0 copies)
    int tg_G = 0, tg_HG = 0;
    DBuf<int4> d_tg_info;
    DBuf<int32_t> d_tg_hrow, d_tg_owner, d_tg_pol, d_tg_cnt0, d_tg_cnt, d_tg_hcnt0, d_tg_hcnt, d_tg_pos0, d_tg_pos,
        d_cls_tcoff, d_cls_tc, d_cls_troff, d_cls_tr;
    DBuf<KpTopoCons> d_cls_tce;
    DBuf<int2> d_tce_hosts;
    DBuf<int2> d_tg_frow;
    DBuf<int32_t> d_tg_late;
    DBuf<uint64_t> d_cls_birth, d_born_s, d_born_m, d_late_sib;
    DBuf<int32_t> d_late_grp;
    int tg_nlate = 0;
    bool tg_var = false;  // variant groups (topo_build): late_sib / late_grp are live
    std::vector<uint64_t> h_late_sib;
    std::vector<uint64_t> h_cls_birth;
    DBuf<KpTopoRec> d_cls_tre;
    DBuf<uint64_t> d_tg_known0, d_tg_known;
    DBuf<uint8_t> d_cls_kneutral, d_vrank;
    // consolidation over topology (kp_consolidate_prepare sets cons_extra before kp_solve_prepare): the candidates'
    // reschedulable pods (node, pod, candidate) join the base counts; cons_dec[candidate][group] = its value-keyed counts
    std::vector<std::array<int, 3>> cons_extra;
    int cons_extra_ncand = 0;
    // ... and the pending pods, in SimulateScheduling's order: with cons_topo set, topo_build picks each topology
    // identity's first owner per probe (pending pods, then the candidates' pods) instead of over the cluster's pods
    std::vector<int> cons_pend;
    bool cons_topo = false;
    std::vector<std::map<int, std::vector<int32_t>>> cons_dec;
    // hostname pod affinity: per candidate, the hostname-affinity groups whose domain on its node holds a selected pod
    // only through the candidate's reschedulable pods (a probe of the candidate has one positive domain less); h_tpos0 =
    // positive domains per group over every bound pod
    std::vector<std::map<int, int>> cons_hdec;
    std::vector<std::vector<int>> cons_hlost;
    std::vector<int32_t> h_tpos0;
    DBuf<int32_t> d_hpos0, d_tg_ha, d_ring_cls, d_ring_shape;
    DBuf<uint32_t> d_g_key;  // HBM slice arrays of node-dense plans (KpDev::g_key ...)
    DBuf<uint16_t> d_g_ord, d_g_last;
    DBuf<uint8_t> d_g_tmpl;
    DBuf<KpDev> d_self;  // device copy of dev for out-of-line kernel helpers (KpDev::self)
    DBuf<KpDev> d_cons_dev;  // device copies of a consolidation launch's tables for the FULL variant (by pointer)
    DBuf<KpCons> d_cons_k;
    std::vector<uint64_t> h_tknown_dg;       // [G] buildDomainGroups' domains (before any pod is counted)
    DBuf<int32_t> d_dec_soff, d_dec_moff, d_dec_g, d_dec_v, d_pt_cnt, d_pt_hd;
    DBuf<uint64_t> d_pt_known, d_pt_dgk;
    std::vector<uint8_t> tg_host_aff;        // [G] hostname pod-affinity group (not in consolidation probes)
    // preference relaxation stages of the prepared solve (expand_preferences) and MIN_VALUES_POLICY
    PrefExpansion pref;
    bool best_effort = false;
    DBuf<int32_t> d_relax_next, d_shape_next, d_pod_cls0, d_pod_shape0, d_last_ep;
    // last results (host)
    int last_N = 0, M = 0;
    std::vector<int32_t> h_nc_tmpl;
};

static kp_status fail(kp_ctx* c, kp_status st, const std::string& msg) {
    if (c) c->err = msg;
    return st;
}
#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) return fail(ctx, KP_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

// Runs f on the ctx and, concurrently (one host thread each), on its peer ctxs.  The primary's status wins; otherwise
// the first failing peer's status is returned with its message.
template <class F>
static kp_status fan_out(kp_ctx* ctx, F f) {
    if (ctx->peers.empty()) return f(ctx);
    const size_t G = ctx->peers.size();
    std::vector<kp_status> st(G, KP_OK);
    std::vector<std::thread> th;
    th.reserve(G);
    for (size_t i = 0; i < G; i++)
        th.emplace_back([&st, &f, ctx, i] {
            try {
                st[i] = f(ctx->peers[i]);
            } catch (...) {  // an exception may not leave the thread (std::terminate)
                st[i] = fail(ctx->peers[i], KP_E_INVALID, "host error");
            }
        });
    const kp_status s0 = f(ctx);
    for (auto& t : th) t.join();
    if (s0 != KP_OK) return s0;
    for (size_t i = 0; i < G; i++)
        if (st[i] != KP_OK)
            return fail(ctx, st[i], "device " + std::to_string(ctx->peers[i]->device) + " (peer " + std::to_string(i + 1) +
                                        "): " + ctx->peers[i]->err);
    return KP_OK;
}

extern "C" const char* kp_version(void) { return "kpsim 0.1 (gfx950)"; }

extern "C" const char* kp_last_error(const kp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

extern "C" kp_status kp_ctx_create(const kp_device_opts* opts, kp_ctx** out) try {
    if (!out) return KP_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return KP_E_DEVICE;
    if (opts && opts->n_devices > 1) {
        // multi-device ctx: the primary is devices[0], each further entry gets a peer ctx (the same ordinal may repeat:
        // two streams on one device)
        if (!opts->devices) return KP_E_INVALID;
        for (int i = 0; i < opts->n_devices; i++)
            if (opts->devices[i] < 0 || opts->devices[i] >= n) return KP_E_DEVICE;
        kp_device_opts one = *opts;
        one.n_devices = 0;
        one.devices = nullptr;
        one.device = opts->devices[0];
        kp_ctx* primary = nullptr;
        kp_status st = kp_ctx_create(&one, &primary);
        if (st != KP_OK) return st;
        for (int i = 1; i < opts->n_devices && st == KP_OK; i++) {
            one.device = opts->devices[i];
            kp_ctx* peer = nullptr;
            st = kp_ctx_create(&one, &peer);
            if (st == KP_OK) primary->peers.push_back(peer);
        }
        if (st != KP_OK) {
            kp_ctx_destroy(primary);
            return st;
        }
        *out = primary;
        return KP_OK;
    }
    auto ctx = std::make_unique<kp_ctx>();
    ctx->device = opts ? opts->device : 0;
    if (opts) {
        if (opts->preference_policy != KP_PREFERENCE_RESPECT && opts->preference_policy != KP_PREFERENCE_IGNORE)
            return KP_E_INVALID;
        ctx->pref_policy = opts->preference_policy;
        ctx->reserved_capacity = opts->reserved_capacity ? 1 : 0;
    }
    if (ctx->device < 0 || ctx->device >= n) return KP_E_DEVICE;
    if (hipSetDevice(ctx->device) != hipSuccess) return KP_E_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, ctx->device) != hipSuccess) return KP_E_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KP_E_DEVICE;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) return KP_E_DEVICE;
    for (auto& e : ctx->ev)
        if (hipEventCreate(&e) != hipSuccess) return KP_E_DEVICE;
    if (kp_ffd_set_attributes() != hipSuccess || kp_cons_set_attributes() != hipSuccess) return KP_E_DEVICE;
    *out = ctx.release();
    return KP_OK;
} catch (...) {
    return KP_E_DEVICE;
}

extern "C" kp_status kp_ctx_destroy(kp_ctx* ctx) {
    if (!ctx) return KP_OK;
    for (kp_ctx* p : ctx->peers) kp_ctx_destroy(p);
    ctx->peers.clear();
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    for (auto& e : ctx->ev)
        if (e) hipEventDestroy(e);
    for (auto& e : ctx->lev)
        if (e) hipEventDestroy(e);
    if (ctx->lstream2) {
        hipStreamSynchronize(ctx->lstream2);
        hipStreamDestroy(ctx->lstream2);
    }
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;  // every DBuf member frees its device memory (on the device set above)
    return KP_OK;
}

// ---------------------------------------------------------------------------------------------
// catalog upload
// ---------------------------------------------------------------------------------------------
static void rebuild_avail(kp_ctx* c, const std::vector<uint8_t>& avail) {
    std::fill(c->avail_zc.begin(), c->avail_zc.end(), 0ull);
    for (size_t o = 0; o < c->off_type.size(); o++)
        if (c->off_slot[o] >= 0 && avail[o]) c->avail_zc[c->off_type[o]] |= 1ull << c->off_slot[o];
}

static kp_status upload_launch_tables(kp_ctx* c, const kp_catalog_view* v, const std::vector<uint8_t>& avail);

// The ResvTab rows, the header with their device pointers, and the per-type spans / capacities / prices.
static hipError_t upload_resv(kp_ctx* c, hipStream_t s) {
    ResvTab& X = c->h_ro;
    X = ResvTab{};
    X.n = (int)c->ro_type.size();
    X.w = (X.n + 63) / 64;
    X.nrid = (int)c->ro_rid_vid.size();
    X.ridw = (X.nrid + 63) / 64;
    X.ctv = c->key_ct >= 0 ? c->cat.keys[c->key_ct].find("reserved") : -1;
    hipError_t e = hipSuccess, first = hipSuccess;  // the first failed upload is returned before the header goes up
    auto up = [&](DBuf<int32_t>& b, const std::vector<int32_t>& v) -> const int32_t* {
        if ((e = b.upload(v, s)) != hipSuccess) {
            if (first == hipSuccess) first = e;
            return nullptr;
        }
        return b.p;
    };
    X.type = up(c->d_ro_type, c->ro_type);
    X.zone = up(c->d_ro_zone, c->ro_zone);
    X.zid = up(c->d_ro_zid, c->ro_zid);
    X.rid = up(c->d_ro_rid, c->ro_rid);
    X.ridv = up(c->d_ro_ridv, c->ro_ridv);
    X.rtype = up(c->d_ro_rtype, c->ro_rtype);
    X.rid_vid = up(c->d_ro_rid_vid, c->ro_rid_vid);
    if (first != hipSuccess) return first;
    if ((e = c->d_ro_avail.upload(c->ro_avail, s)) != hipSuccess) return e;
    X.avail = c->d_ro_avail.p;
    c->h_ro_up.assign(1, X);
    if ((e = c->d_ro.upload(c->h_ro_up, s)) != hipSuccess) return e;
    if ((e = c->d_type_ro.upload(c->type_ro, s)) != hipSuccess) return e;
    std::vector<int32_t> rc = c->rcap0;
    if (rc.empty()) rc.push_back(0);
    if ((e = c->d_rcap0.upload(rc, s)) != hipSuccess) return e;
    std::vector<double> pr = c->ro_price;
    if (pr.empty()) pr.push_back(0.0);
    return c->d_ro_price.upload(pr, s);
}

static kp_status catalog_upload_one(kp_ctx* ctx, const kp_catalog_view* v, uint64_t epoch) try {
    if (!ctx || !v) return KP_E_INVALID;
    // every prepared solve / consolidation pass captured device pointers and sizes of the previous catalog, and the
    // tables below may be reallocated: nothing prepared survives an upload, successful or not
    ctx->have_catalog = false;
    ctx->prepared = ctx->executed = false;
    ctx->cons_prepared = ctx->cons_prep_valid = false;
    ctx->cons_gen++;  // cached pass rows and read-backs of kp_consolidate_command are stale
    HIPCHK(hipSetDevice(ctx->device));
    const int T = v->n_types, R = v->n_resources, KL = v->n_label_keys;
    if (T <= 0 || R <= 0 || R > KP_MAX_R) return fail(ctx, KP_E_INVALID, "bad n_types / n_resources");
    if (T > KP_MAX_TYPES) return fail(ctx, KP_E_UNSUPPORTED, "more than KP_MAX_TYPES instance types");
    kp_ctx* c = ctx;
    c->have_catalog = false;
    c->T = T;
    c->TW = (T + 63) / 64;
    c->R = R;
    c->resource_names.assign(v->resource_names, v->resource_names + R);
    c->type_names.assign(v->type_names, v->type_names + T);
    c->cat = Dicts();
    c->has_reserved = false;
    c->solve_unsupported.clear();
    // label keys (type requirements) then offering keys
    std::vector<int> lk(KL), ok(v->n_offering_keys);
    for (int k = 0; k < KL; k++) lk[k] = c->cat.key(normalize(v->label_keys[k]));
    for (int k = 0; k < v->n_offering_keys; k++) ok[k] = c->cat.key(normalize(v->offering_keys[k]));
    const int Kc = (int)c->cat.keys.size();
    c->Kcat = Kc;
    // type values: state per (t, catalog key)
    std::vector<int8_t> st((size_t)T * Kc, KP_LABEL_ABSENT);
    std::vector<std::vector<int>> tv((size_t)T * Kc);
    std::vector<uint8_t> multi(Kc, 0);
    for (int t = 0; t < T; t++) {
        for (int k = 0; k < KL; k++) {
            const int s = v->label_state[(size_t)t * KL + k];
            const int key = lk[k];
            auto& cell = tv[(size_t)t * Kc + key];
            if (s == KP_LABEL_ABSENT) continue;
            int8_t& stt = st[(size_t)t * Kc + key];
            if (s == KP_LABEL_DOES_NOT_EXIST) {
                if (stt == KP_LABEL_ABSENT) stt = KP_LABEL_DOES_NOT_EXIST;
                continue;
            }
            const int o0 = v->label_offsets[(size_t)t * KL + k], o1 = v->label_offsets[(size_t)t * KL + k + 1];
            std::vector<int> ids;
            for (int i = o0; i < o1; i++) ids.push_back(c->cat.keys[key].id(v->label_values[i]));
            std::sort(ids.begin(), ids.end());
            ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
            cell = ids;
            stt = ids.empty() ? KP_LABEL_DOES_NOT_EXIST : KP_LABEL_IN;
            if (ids.size() > 1) multi[key] = 1;
        }
    }
    // single-valued requirements of each type (Requirement.Len() == 1): instanceToNodeClaim's labels
    c->type_single.assign(T, {});
    for (int t = 0; t < T; t++)
        for (int key = 0; key < Kc; key++)
            if (tv[(size_t)t * Kc + key].size() == 1) c->type_single[t].push_back({key, tv[(size_t)t * Kc + key][0]});
    // offering-role keys are multi-valued on the type side in AWS (zone, capacity-type, ...): treat every key
    // that appears in offerings as multi so their value masks exist
    for (int k = 0; k < v->n_offering_keys; k++) multi[ok[k]] = 1;
    // offering values
    const int O = v->n_offerings, KO = v->n_offering_keys;
    auto role = [&](const char* n) { return c->cat.find_key(n); };
    c->key_zone = role("topology.kubernetes.io/zone");
    c->key_ct = role("karpenter.sh/capacity-type");
    c->key_zoneid = role("topology.k8s.aws/zone-id");
    c->key_resvid = role("karpenter.k8s.aws/capacity-reservation-id");
    c->key_resvtype = role("karpenter.k8s.aws/capacity-reservation-type");
    for (int k = 0; k < KO; k++) {
        const int key = ok[k];
        if (key != c->key_zone && key != c->key_ct && key != c->key_zoneid && key != c->key_resvid &&
            key != c->key_resvtype)
            return fail(ctx, KP_E_UNSUPPORTED, "offering requirement key outside {zone, capacity-type, zone-id, reservation}");
    }
    if (c->key_zone < 0 || c->key_ct < 0) return fail(ctx, KP_E_INVALID, "offerings need zone and capacity-type keys");
    int kz = -1, kc = -1, kzi = -1, kri = -1, krt = -1;
    for (int k = 0; k < KO; k++) {
        if (ok[k] == c->key_zone) kz = k;
        if (ok[k] == c->key_ct) kc = k;
        if (ok[k] == c->key_zoneid) kzi = k;
        if (ok[k] == c->key_resvid) kri = k;
        if (ok[k] == c->key_resvtype) krt = k;
    }
    std::vector<int> zslots, cslots;  // value ids
    std::map<int, int> zone_to_zid;   // zone value id → zone-id value id or -1
    c->off_type.assign(O, 0);
    c->off_slot.assign(O, -1);
    std::vector<int> off_zone(O), off_ct(O);
    std::vector<uint8_t> avail(O);
    std::vector<int> ro_rows;
    for (int o = 0; o < O; o++) {
        const int t = v->offering_type[o];
        if (t < 0 || t >= T) return fail(ctx, KP_E_INVALID, "offering_type out of range");
        c->off_type[o] = t;
        avail[o] = v->offering_available[o] ? 1 : 0;
        auto lab = [&](int k, int& state) -> const char* {
            if (k < 0) {
                state = KP_LABEL_ABSENT;
                return nullptr;
            }
            state = v->offering_label_state[(size_t)o * KO + k];
            return v->offering_label_values[(size_t)o * KO + k];
        };
        int sz, sc, szi, sri, srt;
        const char* z = lab(kz, sz);
        const char* ct = lab(kc, sc);
        const char* zi = lab(kzi, szi);
        lab(kri, sri);
        lab(krt, srt);
        if (sz != KP_LABEL_IN || sc != KP_LABEL_IN) return fail(ctx, KP_E_UNSUPPORTED, "offering without zone / capacity-type");
        if (sri == KP_LABEL_IN || srt == KP_LABEL_IN || !strcmp(ct, "reserved")) {
            // reserved offerings (offering.go:164-194): the ResvTab of Solve and the launch tables; consolidation
            // rejects the catalog
            c->has_reserved = true;
            off_zone[o] = off_ct[o] = -1;
            ro_rows.push_back(o);
            continue;
        }
        if (sri == KP_LABEL_ABSENT || srt == KP_LABEL_ABSENT)
            return fail(ctx, KP_E_UNSUPPORTED, "od/spot offerings must carry reservation keys as DoesNotExist (offering.go:144-145)");
        const int zv = c->cat.keys[c->key_zone].id(z), cv = c->cat.keys[c->key_ct].id(ct);
        int ziv = -1;
        if (szi == KP_LABEL_IN) ziv = c->cat.keys[c->key_zoneid].id(zi);
        else if (szi == KP_LABEL_DOES_NOT_EXIST) return fail(ctx, KP_E_UNSUPPORTED, "zone-id DoesNotExist on an offering");
        auto itz = zone_to_zid.find(zv);
        if (itz == zone_to_zid.end()) zone_to_zid[zv] = ziv;
        else if (itz->second != ziv) return fail(ctx, KP_E_UNSUPPORTED, "zone-id is not a function of zone");
        int zi_ = (int)(std::find(zslots.begin(), zslots.end(), zv) - zslots.begin());
        if (zi_ == (int)zslots.size()) zslots.push_back(zv);
        int ci_ = (int)(std::find(cslots.begin(), cslots.end(), cv) - cslots.begin());
        if (ci_ == (int)cslots.size()) cslots.push_back(cv);
        off_zone[o] = zi_;
        off_ct[o] = ci_;
    }
    const int NZ = (int)zslots.size(), NC = (int)cslots.size();
    if (NZ * NC > KP_MAX_SLOTS) return fail(ctx, KP_E_UNSUPPORTED, "more than 64 zone x capacity-type pools");
    c->n_slots = NZ * NC;
    c->slot_zone.assign(c->n_slots, 0);
    c->slot_ct.assign(c->n_slots, 0);
    c->slot_zoneid.assign(c->n_slots, -1);
    for (int zi_ = 0; zi_ < NZ; zi_++)
        for (int ci_ = 0; ci_ < NC; ci_++) {
            const int s = zi_ * NC + ci_;
            c->slot_zone[s] = zslots[zi_];
            c->slot_ct[s] = cslots[ci_];
            c->slot_zoneid[s] = zone_to_zid[zslots[zi_]];
        }
    c->slot_price.assign((size_t)T * KP_MAX_SLOTS, 1.7976931348623157e308);
    for (int o = 0; o < O; o++) {
        if (off_zone[o] < 0) continue;
        const int s = off_zone[o] * NC + off_ct[o];
        c->off_slot[o] = s;
        c->slot_price[(size_t)c->off_type[o] * KP_MAX_SLOTS + s] = v->offering_price[o];
    }
    c->avail_zc.assign(T, 0);
    rebuild_avail(c, avail);
    // reserved offerings: ResvTab rows ordered by type, each type's rows inside one 64-row word (padding rows between),
    // reservations numbered densely in row order; the ReservationManager's initial capacity per reservation
    // (NewReservationManager: the least ReservationCapacity among the offerings carrying the ID)
    c->ro_ok = true;
    c->ro_why.clear();
    c->ro_type.clear();
    c->ro_zone.clear();
    c->ro_zid.clear();
    c->ro_rid.clear();
    c->ro_ridv.clear();
    c->ro_rtype.clear();
    c->ro_rid_vid.clear();
    c->ro_off.clear();
    c->ro_price.clear();
    c->rcap0.clear();
    c->type_ro.assign(T, 0u);
    if (!ro_rows.empty()) {
        std::stable_sort(ro_rows.begin(), ro_rows.end(), [&](int a, int b) { return c->off_type[a] < c->off_type[b]; });
        std::map<int, int> rid_of;  // reservation-id value id -> reservation
        for (size_t a = 0; a < ro_rows.size() && c->ro_ok;) {
            size_t b = a;
            while (b < ro_rows.size() && c->off_type[ro_rows[b]] == c->off_type[ro_rows[a]]) b++;
            const int cnt = (int)(b - a), t = c->off_type[ro_rows[a]];
            if (cnt > 64) {  // one instance type with more than 64 reservations: its rows do not fit one word
                c->ro_ok = false;
                c->ro_why = std::string("instance type ") + (v->type_names && v->type_names[t] ? v->type_names[t] : "?") +
                            " has more than 64 reserved offerings (one 64-row ResvTab word per type)";
                break;
            }
            while ((c->ro_type.size() % 64) + cnt > 64) {  // padding up to the next word
                c->ro_type.push_back(-1);
                c->ro_zone.push_back(0);
                c->ro_zid.push_back(-1);
                c->ro_rid.push_back(0);
                c->ro_ridv.push_back(0);
                c->ro_rtype.push_back(-1);
                c->ro_off.push_back(-1);
                c->ro_price.push_back(0.0);
            }
            const int first = (int)c->ro_type.size();
            c->type_ro[t] = (uint32_t)(first / 64) << 16 | (uint32_t)(first % 64) << 8 | (uint32_t)cnt;
            for (size_t i = a; i < b; i++) {
                const int o = ro_rows[i];
                auto lab = [&](int k, int& state) -> const char* {
                    state = k < 0 ? KP_LABEL_ABSENT : v->offering_label_state[(size_t)o * KO + k];
                    return k < 0 ? nullptr : v->offering_label_values[(size_t)o * KO + k];
                };
                int sz, sc, szi, sri, srt;
                const char* z = lab(kz, sz);
                const char* ct = lab(kc, sc);
                const char* zi = lab(kzi, szi);
                const char* ri = lab(kri, sri);
                const char* rt = lab(krt, srt);
                if (strcmp(ct, "reserved") != 0 || sri != KP_LABEL_IN)
                    return fail(ctx, KP_E_UNSUPPORTED, "reserved offering without capacity-type reserved / reservation-id");
                const int ridv = c->cat.keys[c->key_resvid].id(ri);
                auto it = rid_of.find(ridv);
                const int rc = v->offering_reservation_capacity ? v->offering_reservation_capacity[o] : 0;
                int r;
                if (it == rid_of.end()) {
                    r = (int)c->ro_rid_vid.size();
                    rid_of[ridv] = r;
                    c->ro_rid_vid.push_back(ridv);
                    c->rcap0.push_back(rc);
                } else {
                    r = it->second;
                    c->rcap0[r] = std::min(c->rcap0[r], rc);
                }
                c->ro_type.push_back(t);
                c->ro_zone.push_back(c->cat.keys[c->key_zone].id(z));
                c->ro_zid.push_back(szi == KP_LABEL_IN ? c->cat.keys[c->key_zoneid].id(zi) : -1);
                c->ro_rid.push_back(r);
                c->ro_ridv.push_back(ridv);
                c->ro_rtype.push_back(srt == KP_LABEL_IN ? c->cat.keys[c->key_resvtype].id(rt) : -1);
                c->ro_off.push_back(o);
                c->ro_price.push_back(v->offering_price[o]);
            }
            a = b;
        }
        if (c->ro_ok && ((int)c->ro_type.size() > KP_MAX_RO || (int)c->ro_rid_vid.size() > KP_MAX_RO)) {
            c->ro_ok = false;
            c->ro_why = "more than KP_MAX_RO (1024) reserved offerings";
        }
        if (!c->ro_ok) {
            for (auto* x : {&c->ro_type, &c->ro_zone, &c->ro_zid, &c->ro_rid, &c->ro_ridv, &c->ro_rtype, &c->ro_rid_vid,
                            &c->ro_off, &c->rcap0})
                x->clear();
            c->ro_price.clear();
            c->type_ro.assign(T, 0u);
        }
    }
    c->ro_avail.assign(std::max<size_t>(1, (c->ro_type.size() + 63) / 64), 0ull);
    for (size_t i = 0; i < c->ro_off.size(); i++)
        if (c->ro_off[i] >= 0 && avail[c->ro_off[i]]) c->ro_avail[i / 64] |= 1ull << (i % 64);
    // multi-valued keys: value masks (<= 64 values)
    c->wide_resvid = false;
    c->resvid_rows = false;
    c->cat_kflags.assign(Kc, 0);
    c->cat_multi.assign(Kc, -1);
    c->n_multi = 0;
    for (int k = 0; k < Kc; k++) {
        bool present = false;
        for (int t = 0; t < T && !present; t++) present = st[(size_t)t * Kc + k] != KP_LABEL_ABSENT;
        if (!present && !multi[k]) continue;  // offering-only key absent from every type
        if (multi[k]) {
            if (c->cat.keys[k].vals.size() > 64) {
                // the Solve tables hold a multi-valued label as a 64-bit value mask; the launch path has no such limit.
                // The reservation-id label (one value per capacity reservation) is exempt: reserved offerings are
                // evaluated through ResvTab, and a type's label values are its ResvTab rows' reservation IDs, so a
                // pod or NodePool requirement on the key is tested per type over those rows (KF_RESV_ROWS, eval_wave)
                // instead of a 64-bit value mask — when every type's label is exactly its rows' IDs (else refused:
                // wide_resvid without resvid_rows)
                if (k == c->key_resvid && c->ro_ok) {
                    c->wide_resvid = true;
                    bool rows_ok = true;
                    for (int t = 0; t < T && rows_ok; t++) {
                        const uint32_t tr = c->type_ro[t];
                        const int r0 = (int)(tr >> 16) * 64 + (int)((tr >> 8) & 0xFF), n = (int)(tr & 0xFF);
                        std::set<int> rows;
                        for (int r = 0; r < n; r++) rows.insert(c->ro_ridv[r0 + r]);
                        const int8_t ls = st[(size_t)t * Kc + k];
                        if (ls == KP_LABEL_IN) {
                            const std::vector<int>& lv = tv[(size_t)t * Kc + k];
                            rows_ok = std::set<int>(lv.begin(), lv.end()) == rows;
                        } else {
                            rows_ok = rows.empty();
                        }
                    }
                    c->resvid_rows = rows_ok;  // the Solve's key layout flags it (KF_RESV_ROWS); no mask, no cat flag
                    continue;
                }
                c->solve_unsupported = k == c->key_resvid && !c->ro_why.empty()
                                           ? c->ro_why
                                           : "multi-valued label " + c->cat.keys[k].name + " with > 64 values";
                continue;
            }
            c->cat_kflags[k] = KF_CAT_MULTI;
            c->cat_multi[k] = c->n_multi++;
        } else {
            c->cat_kflags[k] = KF_CAT_SINGLE;
        }
    }
    const int TW = c->TW;
    std::vector<uint16_t> tval((size_t)Kc * T, VAL_ABSENT);
    std::vector<uint64_t> mmask((size_t)std::max(1, c->n_multi) * T, 0), dne((size_t)Kc * TW, 0);
    c->h_multi_state.assign((size_t)std::max(1, c->n_multi) * T, KP_LABEL_ABSENT);
    for (int k = 0; k < Kc; k++) {
        for (int t = 0; t < T; t++) {
            const int8_t s = st[(size_t)t * Kc + k];
            if (s == KP_LABEL_DOES_NOT_EXIST) dne[(size_t)k * TW + t / 64] |= 1ull << (t % 64);
            if (c->cat_kflags[k] & KF_CAT_SINGLE) {
                if (s == KP_LABEL_DOES_NOT_EXIST) tval[(size_t)k * T + t] = VAL_DNE;
                else if (s == KP_LABEL_IN) tval[(size_t)k * T + t] = (uint16_t)tv[(size_t)t * Kc + k][0];
                if (c->cat.keys[k].vals.size() >= VAL_ABSENT) return fail(ctx, KP_E_UNSUPPORTED, "label dictionary too large");
            } else if (c->cat_kflags[k] & KF_CAT_MULTI) {
                uint64_t m = 0;
                if (s == KP_LABEL_IN)
                    for (int id : tv[(size_t)t * Kc + k]) m |= 1ull << id;
                mmask[(size_t)c->cat_multi[k] * T + t] = m;
                c->h_multi_state[(size_t)c->cat_multi[k] * T + t] = (uint8_t)s;
            }
        }
    }
    c->alloc_rt.assign((size_t)R * T, 0);
    c->cap_rt.assign((size_t)R * T, 0);
    std::vector<uint64_t> nonneg(TW, 0);
    for (int t = 0; t < T; t++) {
        bool nn = true;
        for (int r = 0; r < R; r++) {
            c->alloc_rt[(size_t)r * T + t] = v->allocatable[(size_t)t * R + r];
            c->cap_rt[(size_t)r * T + t] = v->capacity[(size_t)t * R + r];
            nn = nn && v->allocatable[(size_t)t * R + r] >= 0;
        }
        if (nn) nonneg[t / 64] |= 1ull << (t % 64);
    }
    std::vector<int> idx(T);
    for (int t = 0; t < T; t++) idx[t] = t;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return c->type_names[a] < c->type_names[b]; });
    std::vector<uint32_t> rank(T);
    for (int i = 0; i < T; i++) {
        rank[idx[i]] = (i > 0 && c->type_names[idx[i]] == c->type_names[idx[i - 1]]) ? rank[idx[i - 1]] : (uint32_t)i;
    }
    c->h_multi_mask = mmask;
    hipStream_t s = c->stream;
    HIPCHK(c->d_type_val.upload(tval, s));
    HIPCHK(c->d_multi_mask.upload(mmask, s));
    c->multi16_ok = c->n_multi <= 5;
    for (int k = 0; k < Kc; k++)
        if ((c->cat_kflags[k] & KF_CAT_MULTI) && c->cat.keys[k].vals.size() > 16) c->multi16_ok = false;
    if (c->multi16_ok) {
        std::vector<uint16_t> m16(mmask.size());
        for (size_t i = 0; i < mmask.size(); i++) m16[i] = (uint16_t)mmask[i];
        HIPCHK(c->d_multi16.upload(m16, s));
    }
    HIPCHK(c->d_dne_mask.upload(dne, s));
    HIPCHK(c->d_alloc.upload(c->alloc_rt, s));
    HIPCHK(c->d_cap.upload(c->cap_rt, s));
    HIPCHK(c->d_avail_zc.upload(c->avail_zc, s));
    HIPCHK(c->d_slot_price.upload(c->slot_price, s));
    HIPCHK(c->d_slot_zone.upload(c->slot_zone, s));
    HIPCHK(c->d_slot_ct.upload(c->slot_ct, s));
    HIPCHK(c->d_slot_zoneid.upload(c->slot_zoneid, s));
    HIPCHK(c->d_name_rank.upload(rank, s));
    HIPCHK(c->d_nonneg.upload(nonneg, s));
    HIPCHK(upload_resv(c, s));
    {
        kp_status lst = upload_launch_tables(c, v, avail);
        if (lst != KP_OK) return lst;
    }
    HIPCHK(hipStreamSynchronize(s));
    c->epoch = epoch;
    for (auto& kd : c->cat.keys) kd.freeze();  // the catalog dictionaries are complete: index them for lookups
    c->cat.freeze_keys();
    c->have_catalog = true;
    c->prepared = c->executed = false;
    c->cons_prepared = false;
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_catalog_upload(kp_ctx* ctx, const kp_catalog_view* v, uint64_t epoch) try {
    if (!ctx || !v) return KP_E_INVALID;
    return fan_out(ctx, [&](kp_ctx* c) { return catalog_upload_one(c, v, epoch); });
} catch (...) {
    return fail(ctx, KP_E_INVALID, "kp_catalog_upload: host error");
}

static kp_status patch_avail_one(kp_ctx* ctx, const uint8_t* available, int32_t n, uint64_t epoch) {
    if (!ctx || !available) return KP_E_INVALID;
    ctx->cons_prep_valid = false;
    ctx->cons_gen++;  // cached pass rows and read-backs of kp_consolidate_command are stale
    if (!ctx->have_catalog) return fail(ctx, KP_E_STATE, "no catalog");
    if (n != (int)ctx->off_type.size()) return fail(ctx, KP_E_INVALID, "offering count mismatch");
    HIPCHK(hipSetDevice(ctx->device));
    rebuild_avail(ctx, std::vector<uint8_t>(available, available + n));
    HIPCHK(ctx->d_avail_zc.upload(ctx->avail_zc, ctx->stream));
    std::fill(ctx->ro_avail.begin(), ctx->ro_avail.end(), 0ull);
    for (size_t i = 0; i < ctx->ro_off.size(); i++)
        if (ctx->ro_off[i] >= 0 && available[ctx->ro_off[i]]) ctx->ro_avail[i / 64] |= 1ull << (i % 64);
    HIPCHK(ctx->d_ro_avail.upload(ctx->ro_avail, ctx->stream));
    for (int o = 0; o < n; o++) ctx->l_avail[o] = available[o] ? 1 : 0;
    HIPCHK(ctx->d_l_avail.upload(ctx->l_avail, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->epoch = epoch;
    return KP_OK;
}

extern "C" kp_status kp_catalog_patch_avail(kp_ctx* ctx, const uint8_t* available, int32_t n, uint64_t epoch) try {
    if (!ctx || !available) return KP_E_INVALID;
    return fan_out(ctx, [&](kp_ctx* c) { return patch_avail_one(c, available, n, epoch); });
} catch (...) {
    return fail(ctx, KP_E_INVALID, "kp_catalog_patch_avail: host error");
}

static kp_status patch_price_one(kp_ctx* ctx, const int32_t* idx, const double* price, int32_t n, uint64_t epoch) {
    if (!ctx || (n > 0 && (!idx || !price))) return KP_E_INVALID;
    ctx->cons_prep_valid = false;
    ctx->cons_gen++;  // cached pass rows and read-backs of kp_consolidate_command are stale
    if (!ctx->have_catalog) return fail(ctx, KP_E_STATE, "no catalog");
    HIPCHK(hipSetDevice(ctx->device));
    for (int i = 0; i < n; i++) {
        if (idx[i] < 0 || idx[i] >= (int)ctx->off_type.size()) return fail(ctx, KP_E_INVALID, "offering index");
        if (ctx->off_slot[idx[i]] >= 0)
            ctx->slot_price[(size_t)ctx->off_type[idx[i]] * KP_MAX_SLOTS + ctx->off_slot[idx[i]]] = price[i];
        for (size_t r = 0; r < ctx->ro_off.size(); r++)
            if (ctx->ro_off[r] == idx[i]) ctx->ro_price[r] = price[i];  // (padding rows hold -1)
        ctx->l_price[idx[i]] = price[i];
    }
    if (!ctx->ro_price.empty()) HIPCHK(ctx->d_ro_price.upload(ctx->ro_price, ctx->stream));
    HIPCHK(ctx->d_slot_price.upload(ctx->slot_price, ctx->stream));
    HIPCHK(ctx->d_l_price.upload(ctx->l_price, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->epoch = epoch;
    return KP_OK;
}

extern "C" kp_status kp_catalog_patch_price(kp_ctx* ctx, const int32_t* idx, const double* price, int32_t n,
                                            uint64_t epoch) try {
    if (!ctx || (n > 0 && (!idx || !price))) return KP_E_INVALID;
    return fan_out(ctx, [&](kp_ctx* c) { return patch_price_one(c, idx, price, n, epoch); });
} catch (...) {
    return fail(ctx, KP_E_INVALID, "kp_catalog_patch_price: host error");
}

// ---------------------------------------------------------------------------------------------
// solve: prepare (encode + upload)
// ---------------------------------------------------------------------------------------------
static bool build_hreqs(kp_ctx* c, const kp_requirement* rs, int n, std::map<int, HReq>& out, std::string& err) {
    for (int i = 0; i < n; i++) {
        const kp_requirement& r = rs[i];
        if (!r.key || r.op < 0 || r.op > 5) {
            err = "bad requirement";
            return false;
        }
        HReq q;
        q.key = c->sol.key(normalize(r.key));
        q.complement = !(r.op == KP_OP_IN || r.op == KP_OP_DOES_NOT_EXIST);
        if (r.op == KP_OP_IN || r.op == KP_OP_NOT_IN) {
            for (int j = 0; j < r.n_values; j++) q.vals.push_back(c->sol.keys[q.key].id(r.values[j] ? r.values[j] : ""));
            std::sort(q.vals.begin(), q.vals.end());
            q.vals.erase(std::unique(q.vals.begin(), q.vals.end()), q.vals.end());
        }
        if (r.op == KP_OP_GT || r.op == KP_OP_LT) {
            int64_t x = 0;
            go_atoi(r.n_values > 0 && r.values[0] ? r.values[0] : "", x);
            if (r.op == KP_OP_GT) {
                q.has_gt = true;
                q.gt = x;
            } else {
                q.has_lt = true;
                q.lt = x;
            }
        }
        q.has_min = r.min_values >= 0;
        q.minv = r.min_values;
        auto it = out.find(q.key);
        if (it == out.end()) {
            out.emplace(q.key, q);
            continue;
        }
        // Requirements.Add: requirement.Intersection(existing); values filtered after all keys are interned
        HReq& e = it->second;
        HReq o;
        o.key = q.key;
        o.complement = q.complement && e.complement;
        o.has_gt = q.has_gt || e.has_gt;
        o.gt = (q.has_gt && e.has_gt) ? std::max(q.gt, e.gt) : (q.has_gt ? q.gt : e.gt);
        o.has_lt = q.has_lt || e.has_lt;
        o.lt = (q.has_lt && e.has_lt) ? std::min(q.lt, e.lt) : (q.has_lt ? q.lt : e.lt);
        o.has_min = q.has_min || e.has_min;
        o.minv = (q.has_min && e.has_min) ? std::max(q.minv, e.minv) : (q.has_min ? q.minv : e.minv);
        if (o.has_gt && o.has_lt && o.gt >= o.lt) {
            HReq dne;
            dne.key = q.key;
            dne.has_min = o.has_min;
            dne.minv = o.minv;
            it->second = dne;
            continue;
        }
        std::vector<int> vals;
        if (q.complement && e.complement)
            std::set_union(q.vals.begin(), q.vals.end(), e.vals.begin(), e.vals.end(), std::back_inserter(vals));
        else if (q.complement)
            std::set_difference(e.vals.begin(), e.vals.end(), q.vals.begin(), q.vals.end(), std::back_inserter(vals));
        else if (e.complement)
            std::set_difference(q.vals.begin(), q.vals.end(), e.vals.begin(), e.vals.end(), std::back_inserter(vals));
        else
            std::set_intersection(q.vals.begin(), q.vals.end(), e.vals.begin(), e.vals.end(), std::back_inserter(vals));
        o.vals.clear();
        for (int vv : vals) {
            bool ok = true;
            if (o.has_gt || o.has_lt) {
                int64_t x = 0;
                if (!go_atoi(c->sol.keys[q.key].vals[vv].c_str(), x)) ok = false;
                else if ((o.has_gt && o.gt >= x) || (o.has_lt && o.lt <= x)) ok = false;
            }
            if (ok) o.vals.push_back(vv);
        }
        if (!o.complement) o.has_gt = o.has_lt = false;
        it->second = o;
    }
    return true;
}

static bool tolerates(const kp_taint& taint, const kp_toleration* tols, int n) {
    for (int i = 0; i < n; i++) {
        const kp_toleration& t = tols[i];
        const char* te = t.effect ? t.effect : "";
        const char* tk = t.key ? t.key : "";
        if (*te && strcmp(te, taint.effect ? taint.effect : "")) continue;
        if (*tk && strcmp(tk, taint.key ? taint.key : "")) continue;
        if (t.op == KP_TOL_EXISTS) return true;
        if (!strcmp(t.value ? t.value : "", taint.value ? taint.value : "")) return true;
    }
    return false;
}

// ---------------------------------------------------------------------------------------------
// topology encoding ([core] scheduling/topology.go NewTopology, topologygroup.go)
// ---------------------------------------------------------------------------------------------
namespace {
struct HGroup {
    int type = 0, key = -1, owner = -1, skew = 0, mindom = 0, pol = 0, hrow = -1;
    bool host = false, inverse = false;
    std::vector<uint8_t> sel;   // per class: namespace ∈ namespaces ∧ the label selector matches
    std::vector<uint8_t> memb;  // per class: the class owns the group (owner = the first owner, topo_build)
    std::vector<uint8_t> same;  // per class: an owner whose term's semantics equal the first owner's (filter, minDomains)
    int ident = -1;             // TopologyGroup.Hash() identity (topo_build)
};
struct TopoHost {
    std::vector<HGroup> g;
    std::vector<std::vector<int>> cons, rec;  // per class: constraining groups (| self << 30), recording groups
    std::vector<std::vector<int>> neutral;    // per class: keys added to its digest only for narrowing
    int key_host = -1;
    int n_host = 0;
    // groups created by Topology.Update on a relaxed pod (see topo_build): group → its late bit (-1: created by
    // NewTopology whenever a pod owns it), the late bits each class owns; per late bit, the bits of its identity's
    // variant groups (itself alone for a plain late group) and its group
    std::vector<int> g_late;
    std::vector<uint64_t> cls_birth;
    std::vector<uint64_t> late_sib;
    std::vector<int32_t> late_grp;
    bool any_var = false;
    int n_late = 0;
};

// hashstructure (FormatV2, SlicesAsSets) folds a slice by XOR of its elements' hashes: elements that occur an even
// number of times cancel.  The identity string of such a slice keeps the elements of odd multiplicity, sorted.
std::string parity_join(std::vector<std::string> v) {
    std::sort(v.begin(), v.end());
    std::string out;
    for (size_t i = 0; i < v.size();) {
        size_t j = i;
        while (j < v.size() && v[j] == v[i]) j++;
        if ((j - i) & 1) {
            out += v[i];
            out += '\x1f';
        }
        i = j;
    }
    return out;
}

// labels.Selector over pod labels (metav1.LabelSelector: matchLabels as In, matchExpressions In/NotIn/Exists/DNE)
bool selector_matches(const kp_topology_term& t, const kp_pod_class& pc) {
    if (t.n_selector < 0) return false;  // nil selector
    for (int i = 0; i < t.n_selector; i++) {
        const kp_requirement& q = t.selector[i];
        const char* v = nullptr;
        for (int l = 0; l < pc.n_labels; l++)
            if (pc.label_keys[l] && !strcmp(pc.label_keys[l], q.key)) v = pc.label_values[l] ? pc.label_values[l] : "";
        bool in = false;
        for (int j = 0; v && j < q.n_values; j++) in = in || !strcmp(q.values[j] ? q.values[j] : "", v);
        if ((q.op == KP_OP_IN && !in) || (q.op == KP_OP_NOT_IN && in) || (q.op == KP_OP_EXISTS && !v) ||
            (q.op == KP_OP_DOES_NOT_EXIST && v))
            return false;
    }
    return true;
}
const char* ns_of(const kp_pod_class& pc) { return pc.namespace_name ? pc.namespace_name : "default"; }
}  // namespace

// ---------------------------------------------------------------------------------------------
// preferences ([core] scheduling/preferences.go Relax; kpsim.h kp_pod_class).  Every input class becomes a chain of
// effective classes, one per spec state a pod's Relax steps walk through: stage 0 keeps the input class id, further
// stages are appended and linked by relax_next.  The device switches a failed pod to relax_next[class] and re-queues
// it with Queue.Push(pod, relaxed = true).
// ---------------------------------------------------------------------------------------------
static kp_status expand_preferences(const kp_solve_input* in, int pref_policy, PrefExpansion& X, std::string& err) {
    const int C0 = in->n_classes;
    bool tol_pns = false;  // NewScheduler: a NodePool template carries a PreferNoSchedule taint
    for (int i = 0; i < in->n_nodepools; i++)
        for (int j = 0; j < in->nodepools[i].n_taints; j++) {
            const char* e = in->nodepools[i].taints[j].effect;
            tol_pns |= e && !strcmp(e, "PreferNoSchedule");
        }
    struct St {
        int cls, origin, req_first;
        std::vector<int> pnode, paff, panti, spreads;
        bool pns;
    };
    std::vector<St> st;
    bool any = false;
    for (int c = 0; c < C0; c++) {
        const kp_pod_class& pc = in->classes[c];
        St x{c, c, 0, {}, {}, {}, {}, false};
        if ((pc.n_required_terms > 0 && !pc.required_terms) || (pc.n_preferred_terms > 0 && !pc.preferred_terms) ||
            (pc.n_topology > 0 && !pc.topology)) {
            err = "pod class arrays";
            return KP_E_INVALID;
        }
        // newPodRequirements: sort.Slice(preferred, weight desc) in place (unstable beyond 12 terms: Go's pdqsort);
        // later sorts of the sorted slice, and Relax's SliceStable, keep that order
        for (int i = 0; i < pc.n_preferred_terms; i++) x.pnode.push_back(i);
        go_sort_slice((int)x.pnode.size(),
                      [&](int a, int b) { return pc.preferred_terms[x.pnode[a]].weight > pc.preferred_terms[x.pnode[b]].weight; },
                      [&](int a, int b) { std::swap(x.pnode[a], x.pnode[b]); });
        for (int i = 0; i < pc.n_topology; i++) {
            const kp_topology_term& t = pc.topology[i];
            if (t.type == KP_TOPO_SPREAD) {
                x.spreads.push_back(i);
            } else if (t.weight > 0) {
                (t.type == KP_TOPO_AFFINITY ? x.paff : x.panti).push_back(i);
            }
        }
        for (auto* v : {&x.paff, &x.panti})
            std::stable_sort(v->begin(), v->end(), [&](int a, int b) { return pc.topology[a].weight > pc.topology[b].weight; });
        st.push_back(std::move(x));
    }
    X.relax_next.assign(C0, -1);
    for (size_t w = 0; w < st.size(); w++) {
        const St cur = st[w];
        const kp_pod_class& pc = in->classes[cur.origin];
        St nx = cur;
        bool relaxed = true;
        if (pc.n_required_terms - cur.req_first > 1) {
            nx.req_first++;                       // removeRequiredNodeAffinityTerm
        } else if (!cur.paff.empty()) {
            nx.paff.erase(nx.paff.begin());       // removePreferredPodAffinityTerm (heaviest)
        } else if (!cur.panti.empty()) {
            nx.panti.erase(nx.panti.begin());     // removePreferredPodAntiAffinityTerm (heaviest)
        } else if (!cur.pnode.empty()) {
            nx.pnode.erase(nx.pnode.begin());     // removePreferredNodeAffinityTerm (heaviest)
        } else {
            relaxed = false;
            for (size_t i = 0; i < cur.spreads.size() && !relaxed; i++)
                if (pc.topology[cur.spreads[i]].when_unsatisfiable == KP_SCHEDULE_ANYWAY) {
                    nx.spreads[i] = nx.spreads.back();  // removeTopologySpreadScheduleAnyway: swap with the last
                    nx.spreads.pop_back();
                    relaxed = true;
                }
            if (!relaxed && tol_pns && !cur.pns) {
                bool has = false;  // Toleration.MatchToleration of {Exists, effect PreferNoSchedule}
                for (int i = 0; i < pc.n_tolerations; i++) {
                    const kp_toleration& t = pc.tolerations[i];
                    has |= t.op == KP_TOL_EXISTS && (!t.key || !*t.key) && (!t.value || !*t.value) && t.effect &&
                           !strcmp(t.effect, "PreferNoSchedule");
                }
                if (!has) {
                    nx.pns = true;                // toleratePreferNoScheduleTaints
                    relaxed = true;
                }
            }
        }
        if (!relaxed) continue;
        nx.cls = C0 + (int)(st.size() - C0);
        X.relax_next[cur.cls] = nx.cls;
        X.relax_next.push_back(-1);
        st.push_back(std::move(nx));
        any = true;
    }
    const int CX = (int)st.size();
    if (CX + 64 >= 65535) {
        err = "too many pod classes after preference expansion";
        return KP_E_UNSUPPORTED;
    }
    X.classes.assign(CX, kp_pod_class{});
    X.reqs.assign(CX, {});
    X.tols.assign(CX, {});
    X.terms.assign(CX, {});
    X.filt.assign(CX, {});
    X.origin.assign(CX, 0);
    X.n_input = C0;
    for (const St& x : st) X.origin[x.cls] = x.origin;
    X.strict.assign(CX, {});
    X.has_strict.assign(CX, 0);
    static const kp_toleration pns_tol = {"", KP_TOL_EXISTS, "", "PreferNoSchedule"};
    for (const St& x : st) {
        const kp_pod_class& pc = in->classes[x.origin];
        kp_pod_class& o = X.classes[x.cls];
        o = pc;
        auto& rq = X.reqs[x.cls];
        rq.assign(pc.requirements, pc.requirements + pc.n_requirements);
        if (pc.n_required_terms > 0) {
            const kp_node_selector_term& t = pc.required_terms[x.req_first];
            rq.insert(rq.end(), t.requirements, t.requirements + t.n_requirements);
        }
        auto& fl = X.filt[x.cls];
        if (pc.n_required_terms == 0) {
            fl.emplace_back(pc.requirements, pc.requirements + pc.n_requirements);
        } else {
            for (int i = x.req_first; i < pc.n_required_terms; i++) {
                const kp_node_selector_term& t = pc.required_terms[i];
                fl.emplace_back(pc.requirements, pc.requirements + pc.n_requirements);
                fl.back().insert(fl.back().end(), t.requirements, t.requirements + t.n_requirements);
            }
        }
        if (pref_policy == KP_PREFERENCE_RESPECT && !x.pnode.empty()) {
            X.strict[x.cls] = rq;
            X.has_strict[x.cls] = 1;
            const kp_node_selector_term& t = pc.preferred_terms[x.pnode[0]];
            rq.insert(rq.end(), t.requirements, t.requirements + t.n_requirements);
        }
        auto& tl = X.tols[x.cls];
        tl.assign(pc.tolerations, pc.tolerations + pc.n_tolerations);
        if (x.pns) tl.push_back(pns_tol);
        auto& tm = X.terms[x.cls];
        auto keep = [&](int i) {
            const kp_topology_term& t = pc.topology[i];
            const bool pref = t.type == KP_TOPO_SPREAD ? t.when_unsatisfiable == KP_SCHEDULE_ANYWAY : t.weight > 0;
            if (!(pref && pref_policy == KP_PREFERENCE_IGNORE)) tm.push_back(t);
        };
        for (int i : x.spreads) keep(i);
        for (int i = 0; i < pc.n_topology; i++)
            if (pc.topology[i].type != KP_TOPO_SPREAD && pc.topology[i].weight <= 0) keep(i);
        for (int i : x.paff) keep(i);
        for (int i : x.panti) keep(i);
        o.n_required_terms = o.n_preferred_terms = 0;
        o.required_terms = o.preferred_terms = nullptr;
    }
    for (int c = 0; c < CX; c++) {
        kp_pod_class& o = X.classes[c];
        o.n_requirements = (int32_t)X.reqs[c].size();
        o.requirements = X.reqs[c].data();
        o.n_tolerations = (int32_t)X.tols[c].size();
        o.tolerations = X.tols[c].data();
        o.n_topology = (int32_t)X.terms[c].size();
        o.topology = X.terms[c].data();
    }
    if (!any) X.relax_next.clear();
    X.in = *in;
    X.in.n_classes = CX;
    X.in.classes = X.classes.data();
    return KP_OK;
}

// topo_birth (kp_eval.h) on the host: the late bits `add` are born unless a variant sibling already is (sib empty: no
// variant groups)
static uint64_t late_birth(const std::vector<uint64_t>& sib, uint64_t born, uint64_t add) {
    if (sib.empty()) return born | add;
    for (uint64_t x = add & ~born; x; x &= x - 1) {
        const int b = __builtin_ctzll(x);
        if (!(born & sib[b])) born |= 1ull << b;
    }
    return born;
}

// Topology groups ([core] scheduling/topology.go Update / updateInverseAntiAffinity, topologygroup.go Hash): Go keeps
// one group per TopologyGroup.Hash() — topology key, type, namespaces, label selector, maxSkew and the node filter
// (MakeTopologyNodeFilter: the requirement key sets of the nodeSelector with each required term, the policies, the
// tolerations); hashstructure skips unexported fields, so requirement values and minDomains are not part of it.  Here
// every (class, term) of one identity is one group owned by all those classes, with the first owner's node filter,
// minDomains and selector (see the owner choice below).  A group is created by NewTopology when a pod that owns it is in the batch, or by Topology.Update when a pod relaxes
// into a spec that owns it (countDomains then counts only the bound pods): an identity that only a relaxed stage can
// own — its other owners do not include that stage's input class — is "late", born on the device when the first pod
// relaxes into an owner (at most 64 such identities).  Interns the topology keys.
static kp_status topo_build(kp_ctx* c, const kp_solve_input* in, const std::vector<std::map<int, HReq>>& creq,
                            const std::vector<std::vector<std::map<int, HReq>>>& cfilt, TopoHost& th, std::string& err) {
    const int C = in->n_classes;
    const PrefExpansion& X = c->pref;
    th = TopoHost();
    th.cons.assign(C, {});
    th.rec.assign(C, {});
    th.neutral.assign(C, {});
    struct TEnt {  // one (class, term[, inverse]) owner of an identity
        int cls = 0;
        std::string sig;  // the semantics Hash() does not see: selection, minDomains, Honor filter values / tolerations
        HGroup g;
    };
    std::vector<TEnt> ents;
    std::vector<std::vector<int>> by_ident;  // identity → its entries, class order
    std::map<std::string, int> idents;       // identity → index
    auto hreq_str = [](const HReq& q) {
        std::string r = std::to_string(q.key) + (q.complement ? "!" : "=");
        for (int v : q.vals) r += std::to_string(v) + ",";
        if (q.has_gt) r += ">" + std::to_string(q.gt);
        if (q.has_lt) r += "<" + std::to_string(q.lt);
        return r;
    };
    auto tol_str = [](const kp_toleration& t) {
        return std::string(t.key ? t.key : "") + "\x1d" + std::to_string(t.op) + "\x1d" + (t.value ? t.value : "") + "\x1d" +
               (t.effect ? t.effect : "");
    };
    for (int i = 0; i < C; i++) {
        const kp_pod_class& pc = in->classes[i];
        for (int q = 0; q < pc.n_topology; q++) {
            const kp_topology_term& x = pc.topology[q];
            if (x.type < KP_TOPO_SPREAD || x.type > KP_TOPO_ANTI_AFFINITY || !x.topology_key) {
                err = "bad topology term";
                return KP_E_INVALID;
            }
            // preferred terms reach here only under PREFERENCE_POLICY=Respect (expand_preferences drops them under
            // Ignore): they constrain like required ones until the pod's Relax removes them
            const bool preferred = x.type == KP_TOPO_SPREAD ? x.when_unsatisfiable == KP_SCHEDULE_ANYWAY : x.weight > 0;
            if (preferred && c->pref_policy == KP_PREFERENCE_IGNORE) continue;
            if (x.type == KP_TOPO_SPREAD && x.max_skew <= 0) {
                err = "maxSkew must be positive";
                return KP_E_INVALID;
            }
            for (int j = 0; j < x.n_selector; j++)
                if (!x.selector[j].key || x.selector[j].op < KP_OP_IN || x.selector[j].op > KP_OP_DOES_NOT_EXIST) {
                    err = "label selector operators are In / NotIn / Exists / DoesNotExist";
                    return KP_E_INVALID;
                }
            const std::string nkey = normalize(x.topology_key);
            const int key = c->sol.key(nkey);
            const bool spread = x.type == KP_TOPO_SPREAD;
            // identity fields shared by the forward and inverse group
            std::set<std::string> nss;
            if (spread || x.n_namespaces <= 0) nss.insert(ns_of(pc));
            else
                for (int n = 0; n < x.n_namespaces; n++) nss.insert(x.namespaces[n] ? x.namespaces[n] : "");
            std::string base = std::to_string(x.type) + "\x1e" + nkey + "\x1e";
            for (auto& n : nss) base += n + "\x1f";
            base += "\x1e";
            if (x.n_selector < 0) {
                base += "nil";
            } else {
                std::vector<std::string> el;
                for (int j = 0; j < x.n_selector; j++) {
                    const kp_requirement& r = x.selector[j];
                    std::vector<std::string> vs;
                    for (int v = 0; v < r.n_values; v++) vs.push_back(r.values[v] ? r.values[v] : "");
                    el.push_back(std::string(r.key) + "\x1d" + std::to_string(r.op) + "\x1d" + parity_join(vs));
                }
                base += "sel" + parity_join(el);
            }
            base += "\x1e" + std::to_string(spread ? x.max_skew : INT32_MAX) + "\x1e";
            std::vector<uint8_t> sel(C, 0);
            for (int o = 0; o < C; o++) {
                const kp_pod_class& oc = in->classes[o];
                bool ns_ok = false;
                if (spread || x.n_namespaces <= 0) ns_ok = !strcmp(ns_of(oc), ns_of(pc));
                else
                    for (int n = 0; n < x.n_namespaces; n++) ns_ok = ns_ok || (x.namespaces[n] && !strcmp(x.namespaces[n], ns_of(oc)));
                sel[o] = ns_ok && selector_matches(x, oc);
            }
            const int pol = spread ? (x.node_affinity_policy == KP_POLICY_HONOR ? 1 : 0) | (x.node_taints_policy == KP_POLICY_HONOR ? 2 : 0) : 0;
            for (int inv = 0; inv < 2; inv++) {
                if (inv && (x.type != KP_TOPO_ANTI_AFFINITY || preferred)) break;  // inverse: required anti-affinity only
                std::string id = (inv ? "I\x1e" : "F\x1e") + base;
                std::string sig = std::to_string(spread && x.min_domains > 0 ? x.min_domains : 0) + "\x1e";
                for (uint8_t b : sel) sig += (char)('0' + b);
                if (spread) {  // the node filter (a forward group: spreads have no inverse group)
                    std::vector<std::string> ks;
                    for (auto& f : X.filt[i]) {
                        std::set<std::string> keys;
                        for (auto& r : f)
                            if (r.key) keys.insert(normalize(r.key));
                        std::string k;
                        for (auto& kk : keys) k += kk + "\x1c";
                        ks.push_back(k);
                    }
                    std::vector<std::string> tl;
                    for (int t = 0; t < pc.n_tolerations; t++) tl.push_back(tol_str(pc.tolerations[t]));
                    id += parity_join(ks) + "\x1e" + std::to_string(pol) + "\x1e" + parity_join(tl);
                    if (pol & 1) {  // filter values: one requirement set per filter row, ORed
                        std::set<std::string> rows;
                        for (auto& m : cfilt[i]) {
                            std::string r;
                            for (auto& kv : m) r += hreq_str(kv.second) + ";";
                            rows.insert(r);
                        }
                        sig += "\x1e";
                        for (auto& r : rows) sig += r + "|";
                    }
                    if (pol & 2) {
                        std::set<std::string> ts(tl.begin(), tl.end());
                        sig += "\x1e";
                        for (auto& t : ts) sig += t + "|";
                    }
                }
                auto iit = idents.find(id);
                const int ident = iit != idents.end() ? iit->second : (int)idents.size();
                if (iit == idents.end()) {
                    idents[id] = ident;
                    by_ident.emplace_back();
                }
                // a pod whose terms repeat an identity owns the group its first such term creates (the later ones
                // only AddOwner): one entry per class
                if (!by_ident[ident].empty() && ents[by_ident[ident].back()].cls == i) continue;
                TEnt e;
                e.cls = i;
                e.sig = std::move(sig);
                e.g.type = x.type;
                e.g.key = key;
                e.g.inverse = inv == 1;
                e.g.owner = i;
                e.g.skew = spread ? x.max_skew : INT32_MAX;
                e.g.mindom = spread && x.min_domains > 0 ? x.min_domains : 0;
                e.g.pol = pol;
                e.g.sel = sel;
                e.g.ident = ident;
                by_ident[ident].push_back((int)ents.size());
                ents.push_back(std::move(e));
            }
        }
    }
    if (ents.empty()) return KP_OK;
    const int NI = (int)idents.size();
    const int C0 = X.n_input;
    // One group per identity, as Topology.Update keeps topologyGroups[hash]: the group is the first owner's
    // TopologyGroup (its node filter, minDomains and selector), every later owner only AddOwner()s.  NewTopology
    // iterates its pods in input order, so the first owner is the class of the first input pod whose spec owns the
    // identity; consolidation probes each run their own NewTopology over the pending pods, then their candidates' pods.
    // When the owners' semantics agree any owner is that group.  An identity that only relaxed pods create (no pod of the
    // Solve, or of any probe, owns it at NewTopology) takes the semantics of whichever pod relaxes into it first: it
    // becomes one "variant" group per distinct semantics, each with a late bit of its own; the first relaxation births
    // its variant only (topo_birth: KpDev.late_sib), and the class caches of every owner route the identity's
    // constraint to the born variant (fill_class_cache).  A first owner that differs between consolidation probes, or a
    // probe-dependent mix of NewTopology and relaxation owners, is refused.
    std::vector<uint8_t> gvar;  // per device group: a variant group
    {
        const int P = in->pods.n_pods;
        std::vector<int64_t> firstpos(std::max(C, 1), INT64_MAX);  // Solve: first input pod per stage-0 class
        if (!c->cons_topo) {
            for (int p = P - 1; p >= 0; p--) firstpos[in->pods.class_id[p]] = p;
        } else {
            for (int q = (int)c->cons_pend.size() - 1; q >= 0; q--) firstpos[in->pods.class_id[c->cons_pend[q]]] = q;
        }
        int amb = 0, nvar = 0;
        for (int I = 0; I < NI; I++) {
            const std::vector<int>& es = by_ident[I];
            bool one = true;
            for (int e : es) one = one && ents[e].sig == ents[es[0]].sig;
            int own = es[0];
            bool variant = false;
            auto first_by = [&](const std::vector<int64_t>& pos) {  // the stage-0 owner entry of the smallest position
                int b = -1;
                for (int e : es)
                    if (ents[e].cls < C0 && pos[ents[e].cls] != INT64_MAX && (b < 0 || pos[ents[e].cls] < pos[ents[b].cls])) b = e;
                return b;
            };
            // variants need equal selection (Counts); inverse and affinity groups have no node filter or minDomains, so
            // their semantics differ only in selection
            auto variants_ok = [&]() {
                for (int e : es)
                    if (ents[e].g.inverse || ents[e].g.type != KP_TOPO_SPREAD || ents[e].g.sel != ents[es[0]].g.sel) return false;
                return true;
            };
            if (!one) {
                amb++;
                std::vector<int> relaxed;  // owners that only a relaxation reaches (a stage past 0)
                for (int e : es)
                    if (ents[e].cls >= C0) relaxed.push_back(e);
                auto relaxed_agree = [&](const std::string& s) {
                    for (int e : relaxed)
                        if (ents[e].sig != s) return false;
                    return true;
                };
                const int b = first_by(firstpos);
                int got = -1;
                bool missing = false, same = true;
                if (b < 0 && c->cons_topo) {
                    // consolidation: each probe's first owner is the first of its candidates' pods owning it
                    std::vector<int64_t> cpos(std::max(C, 1), INT64_MAX);
                    int prev = -1;
                    auto close_cand = [&]() {
                        if (prev < 0) return;
                        const int f = first_by(cpos);
                        if (f < 0) missing = true;
                        else if (got < 0) got = f;
                        else same = same && ents[f].sig == ents[got].sig;
                        std::fill(cpos.begin(), cpos.end(), INT64_MAX);
                    };
                    int posq = 0;
                    for (auto& ex : c->cons_extra) {
                        if (ex[2] != prev) {
                            close_cand();
                            prev = ex[2];
                            posq = 0;
                        }
                        const int cl = in->pods.class_id[ex[1]];
                        if (cpos[cl] == INT64_MAX) cpos[cl] = posq;
                        posq++;
                    }
                    close_cand();
                    for (int ci = 0, seen = 0; ci < c->cons_extra_ncand && !missing; ci++) {  // candidates without pods
                        bool has = false;
                        for (; seen < (int)c->cons_extra.size() && c->cons_extra[seen][2] == ci; seen++) has = true;
                        missing = missing || !has;
                    }
                }
                if (b >= 0) {
                    own = b;  // every Solve / probe creates it from this pod at NewTopology
                } else if (got >= 0 && same && !(missing && !relaxed_agree(ents[got].sig))) {
                    own = got;  // every probe that creates it has a first owner of these semantics
                } else if (got >= 0) {
                    // the first owner differs between probes (or some probe's relaxation creates it): one variant per
                    // semantics, each probe starting with its own first owner's variant born (kp_consolidate_prepare)
                    if (!variants_ok()) {
                        err = "topology groups of one TopologyGroup.Hash() identity with different selections whose "
                              "first owner differs between consolidation probes";
                        return KP_E_UNSUPPORTED;
                    }
                    variant = true;
                } else if (!relaxed.empty() && !relaxed_agree(ents[relaxed[0]].sig)) {
                    // no pod owns it at NewTopology: the first relaxation into it decides
                    if (!variants_ok()) {
                        err = "topology groups of one TopologyGroup.Hash() identity with different selections that only "
                              "relaxed pods create";
                        return KP_E_UNSUPPORTED;
                    }
                    variant = true;
                } else if (!relaxed.empty()) {
                    own = relaxed[0];
                }
            }
            if (!variant) {
                HGroup g = ents[own].g;
                g.memb.assign(C, 0);
                g.same.assign(C, 0);
                for (int e : es) {
                    g.memb[ents[e].cls] = 1;
                    g.same[ents[e].cls] |= ents[e].sig == ents[own].sig;
                }
                th.g.push_back(std::move(g));
                gvar.push_back(0);
                continue;
            }
            std::vector<int> done(es.size(), 0);
            for (size_t i = 0; i < es.size(); i++) {  // one group per distinct semantics, its owners the classes holding it
                if (done[i]) continue;
                HGroup g = ents[es[i]].g;
                g.memb.assign(C, 0);
                for (size_t j = i; j < es.size(); j++)
                    if (ents[es[j]].sig == ents[es[i]].sig) {
                        g.memb[ents[es[j]].cls] = 1;
                        done[j] = 1;
                    }
                g.same = g.memb;
                th.g.push_back(std::move(g));
                gvar.push_back(1);
                nvar++;
            }
        }
        if (getenv("KPSIM_DIAG_IDENT"))  // diagnostics: identities whose owners' semantics differ
            fprintf(stderr, "[kpsim] topology identities %d, owner entries %zu, identities with several semantics %d, "
                    "variant groups %d\n", NI, ents.size(), amb, nvar);
    }
    // late identities: a relaxed stage owns it and its input class does not; every variant group is late
    std::vector<std::vector<uint8_t>> own0(NI);  // identity → input classes owning it at stage 0
    for (auto& own : own0) own.assign(std::max(C0, 1), 0);
    for (const HGroup& g : th.g)
        for (int o = 0; o < C && o < C0; o++)
            if (g.memb[o]) own0[g.ident][o] = 1;
    th.g_late.assign(th.g.size(), -1);
    th.late_sib.clear();
    th.late_grp.clear();
    auto new_bit = [&](int gi) -> bool {
        if (th.n_late >= 64) {
            err = "more than 64 topology groups that only relaxed pods own";
            return false;
        }
        th.g_late[gi] = th.n_late++;
        th.late_sib.push_back(1ull << th.g_late[gi]);
        th.late_grp.push_back(gi);
        return true;
    };
    for (int gi = 0; gi < (int)th.g.size(); gi++) {
        const HGroup& g = th.g[gi];
        if (gvar[gi]) {
            if (!new_bit(gi)) return KP_E_UNSUPPORTED;
            continue;
        }
        for (int o = C0; o < C; o++)
            if (g.memb[o] && !own0[g.ident][X.origin[o]]) {
                if (!new_bit(gi)) return KP_E_UNSUPPORTED;
                break;
            }
    }
    for (int gi = 0; gi < (int)th.g.size(); gi++)  // variant siblings: the late bits of one identity's variant groups
        if (gvar[gi])
            for (int gj = 0; gj < (int)th.g.size(); gj++)
                if (gvar[gj] && th.g[gj].ident == th.g[gi].ident) th.late_sib[th.g_late[gi]] |= 1ull << th.g_late[gj];
    th.any_var = false;
    for (uint8_t v : gvar) th.any_var = th.any_var || v;
    th.cls_birth.assign(C, 0);
    for (int gi = 0; gi < (int)th.g.size(); gi++)
        if (th.g_late[gi] >= 0)
            for (int o = 0; o < C; o++)
                if (th.g[gi].memb[o]) th.cls_birth[o] |= 1ull << th.g_late[gi];
    th.key_host = c->sol.key("kubernetes.io/hostname");
    for (int gi = 0; gi < (int)th.g.size(); gi++) {
        HGroup& g = th.g[gi];
        g.host = g.key == th.key_host;
        if (g.host) g.hrow = th.n_host++;
        for (int o = 0; o < C; o++) {
            if (g.inverse) {
                if (g.sel[o]) th.cons[o].push_back(gi | (g.sel[o] << 30));
                if (g.memb[o]) th.rec[o].push_back(gi);
            } else {
                if (g.memb[o]) th.cons[o].push_back(gi | (g.sel[o] << 30));
                if (g.sel[o]) th.rec[o].push_back(gi);
            }
        }
    }
    if (getenv("KPSIM_DIAG_IDENT")) {  // diagnostics: the most constraining / counting groups of one class
        size_t mc = 0, mr = 0;
        for (int o = 0; o < C; o++) mc = std::max(mc, th.cons[o].size()), mr = std::max(mr, th.rec[o].size());
        fprintf(stderr, "[kpsim] topology groups per class: constraining <= %zu, counting <= %zu\n", mc, mr);
    }
    for (int o = 0; o < C; o++) {
        if (th.cons[o].size() > KP_MAX_TOPO || th.rec[o].size() > KP_MAX_TOPO_REC) {
            err = "a pod class is constrained or counted by too many topology groups";
            return KP_E_UNSUPPORTED;
        }
        // constraining entries past the class cache's KP_CC_TC are read from cls_tc as they are: no variant there
        for (size_t q = KP_CC_TC; q < th.cons[o].size(); q++)
            if (gvar[th.cons[o][q] & 0x3FFFFFFF]) {
                err = "a pod class constrained by more than 16 topology groups, one of them a variant group";
                return KP_E_UNSUPPORTED;
            }
        std::set<int> vkeys;  // topo_narrow intersects the groups' domains per value-keyed key
        for (int e : th.cons[o])
            if (!th.g[e & 0x3FFFFFFF].host) vkeys.insert(th.g[e & 0x3FFFFFFF].key);
        if (vkeys.size() > KP_MAX_TOPO_KEYS) {
            err = "a pod class constrained on more than 8 value-keyed topology keys";
            return KP_E_UNSUPPORTED;
        }
        for (int e : th.cons[o]) {
            const HGroup& g = th.g[e & 0x3FFFFFFF];
            if (!g.host && !creq[o].count(g.key) &&
                std::find(th.neutral[o].begin(), th.neutral[o].end(), g.key) == th.neutral[o].end())
                th.neutral[o].push_back(g.key);
        }
    }
    return KP_OK;
}

// KPSIM_PREP_TIMES (diagnostics): host prepare phase times to stderr
static thread_local std::chrono::steady_clock::time_point g_prep_t;
#define PREP_MARK(i)                                                                                          \
    do {                                                                                                      \
        if (getenv("KPSIM_PREP_TIMES")) {                                                                     \
            const auto _n = std::chrono::steady_clock::now();                                                 \
            fprintf(stderr, "[prep] mark %d: %.3f ms\n", i, std::chrono::duration<double>(_n - g_prep_t).count() * 1e3); \
            g_prep_t = _n;                                                                                    \
        }                                                                                                     \
    } while (0)
extern "C" kp_status kp_solve_prepare(kp_ctx* ctx, const kp_solve_input* in) try {
    g_prep_t = std::chrono::steady_clock::now();
    if (!ctx || !in) return KP_E_INVALID;
    ctx->cons_prep_valid = false;
    ctx->cons_gen++;  // cached pass rows and read-backs of kp_consolidate_command are stale
    if (!ctx->have_catalog) return fail(ctx, KP_E_STATE, "kp_solve before kp_catalog_upload");
    if (!ctx->solve_unsupported.empty()) return fail(ctx, KP_E_UNSUPPORTED, "Solve: " + ctx->solve_unsupported);
    if (ctx->has_reserved && !ctx->ro_ok)
        return fail(ctx, KP_E_UNSUPPORTED, "Solve over this catalog: " + ctx->ro_why);
    const auto t0 = clk::now();
    HIPCHK(hipSetDevice(ctx->device));
    kp_ctx* c = ctx;
    c->prepared = c->executed = false;
    c->cons_prepared = false;
    c->any_min_values = false;
    c->min_multi = false;
    if (in->min_values_policy != KP_MIN_VALUES_STRICT && in->min_values_policy != KP_MIN_VALUES_BEST_EFFORT)
        return fail(ctx, KP_E_INVALID, "unknown MIN_VALUES_POLICY");
    c->best_effort = in->min_values_policy == KP_MIN_VALUES_BEST_EFFORT;
    if (in->n_classes < 0 || (in->n_classes > 0 && !in->classes)) return fail(ctx, KP_E_INVALID, "pod classes");
    for (int i = 0; i < in->pods.n_pods; i++)
        if (in->pods.class_id[i] < 0 || in->pods.class_id[i] >= in->n_classes)
            return fail(ctx, KP_E_INVALID, "pod class out of range");
    {
        std::string perr;
        kp_status pst = expand_preferences(in, c->pref_policy, c->pref, perr);
        if (pst != KP_OK) return fail(ctx, pst, perr);
    }
    in = &c->pref.in;  // from here on: the expanded classes (stage 0 of input class i is class i)
    const int T = c->T, TW = c->TW, R = c->R, P = in->pods.n_pods, C = in->n_classes;
    PREP_MARK(0);
    // ---- dictionaries: catalog ∪ solve strings ----
    c->sol = c->cat;
    std::vector<std::map<int, HReq>> creq(C);
    std::string err;
    for (int i = 0; i < C; i++)
        if (!build_hreqs(c, in->classes[i].requirements, in->classes[i].n_requirements, creq[i], err)) return fail(ctx, KP_E_INVALID, err);
    // spread node filters of classes with a nodeAffinityPolicy Honor spread, and strict requirements (podDomains) of
    // classes whose requirements carry a preferred node-affinity term (expand_preferences)
    std::vector<std::vector<std::map<int, HReq>>> cfilt(C);
    std::vector<std::map<int, HReq>> cstrict(C);
    for (int i = 0; i < C; i++) {
        bool honor = false;
        for (int q = 0; q < in->classes[i].n_topology; q++)
            honor |= in->classes[i].topology[q].type == KP_TOPO_SPREAD &&
                     in->classes[i].topology[q].node_affinity_policy == KP_POLICY_HONOR;
        if (honor && c->pref.filt[i].size() > 64)
            return fail(ctx, KP_E_UNSUPPORTED, "a nodeAffinityPolicy Honor spread with more than 64 node-filter terms");
        if (honor)
            for (auto& f : c->pref.filt[i]) {
                cfilt[i].emplace_back();
                if (!build_hreqs(c, f.data(), (int)f.size(), cfilt[i].back(), err)) return fail(ctx, KP_E_INVALID, err);
            }
        if (c->pref.has_strict[i] &&
            !build_hreqs(c, c->pref.strict[i].data(), (int)c->pref.strict[i].size(), cstrict[i], err))
            return fail(ctx, KP_E_INVALID, err);
    }
    // templates: NodePools ordered by weight desc, name asc ([core] NodePoolList.OrderByWeight)
    std::vector<int> npo(in->n_nodepools);
    for (int i = 0; i < in->n_nodepools; i++) npo[i] = i;
    std::sort(npo.begin(), npo.end(), [&](int a, int b) {
        if (in->nodepools[a].weight != in->nodepools[b].weight) return in->nodepools[a].weight > in->nodepools[b].weight;
        return strcmp(in->nodepools[a].name, in->nodepools[b].name) < 0;
    });
    const int NT = (int)npo.size();
    if (NT > KP_MAX_NP) return fail(ctx, KP_E_UNSUPPORTED, "more than 63 NodePools");
    if (C + NT >= 65535) return fail(ctx, KP_E_UNSUPPORTED, "too many pod classes");
    std::vector<std::map<int, HReq>> treq(NT);
    for (int j = 0; j < NT; j++) {
        const kp_nodepool& np = in->nodepools[npo[j]];
        if (!build_hreqs(c, np.requirements, np.n_requirements, treq[j], err)) return fail(ctx, KP_E_INVALID, err);
    }
    for (int i = 0; i < C; i++)
        for (auto& kv : creq[i])
            if (kv.second.has_min) return fail(ctx, KP_E_INVALID, "pod requirements cannot carry minValues");
    if (c->wide_resvid) {  // see catalog_upload_one: no per-type value masks for a reservation-id label this wide
        for (int i = 0; i < C && !c->resvid_rows; i++)
            if (creq[i].count(c->key_resvid))
                return fail(ctx, KP_E_UNSUPPORTED, "a pod requirement on capacity-reservation-id over more than 64 reservations "
                                                   "whose labels are not the types' reserved offerings");
        for (int j = 0; j < NT; j++) {
            auto it = treq[j].find(c->key_resvid);
            if (it == treq[j].end()) continue;
            if (!c->resvid_rows)
                return fail(ctx, KP_E_UNSUPPORTED, "a NodePool requirement on capacity-reservation-id over more than 64 "
                                                   "reservations whose labels are not the types' reserved offerings");
            if (it->second.has_min)  // minValues counts distinct values per type through 64-bit masks
                return fail(ctx, KP_E_UNSUPPORTED, "minValues on capacity-reservation-id over more than 64 reservations");
        }
    }
    TopoHost th;
    {
        const kp_status ts = topo_build(c, in, creq, cfilt, th, err);
        if (ts != KP_OK) return fail(ctx, ts, err);
    }
    // existing nodes (ExistingNode, [core] scheduling/existingnode.go NewExistingNode): requirements =
    // NewLabelRequirements(node labels) + hostname In [name].  Only label keys some pod class constrains can
    // influence Compatible (it iterates the pod's keys), so only those are interned.
    const int E = in->n_existing;
    const int hostname_key = c->sol.find_key("kubernetes.io/hostname");
    std::vector<std::vector<std::pair<int, int>>> exlab(E);  // (key, value id) per node
    for (int j = 0; j < E; j++) {
        const kp_existing_node& en = in->existing[j];
        if (!en.available) return fail(ctx, KP_E_INVALID, "existing node without available resources");
        for (int l = 0; l < en.n_labels; l++) {
            const int k = c->sol.find_key(normalize(en.label_keys[l]));
            if (k < 0 || k == hostname_key) continue;
            exlab[j].push_back({k, c->sol.keys[k].id(en.label_values[l] ? en.label_values[l] : "")});
        }
        if (hostname_key >= 0) exlab[j].push_back({hostname_key, c->sol.keys[hostname_key].id(en.name ? en.name : "")});
    }
    std::map<int, int> host_node;  // hostname value id → existing node
    if (hostname_key >= 0)
        for (int j = E - 1; j >= 0; j--) host_node[exlab[j].back().second] = j;
    const int K = (int)c->sol.keys.size();
    if (K > KP_MAX_KEYS) return fail(ctx, KP_E_UNSUPPORTED, "too many label keys");
    // ExistingNode.Add's requirement merge only changes a node when a NotIn / DoesNotExist pod requirement meets a key
    // the node lacks (a node's labels are single values, which a compatible merge leaves as they are), and that change
    // only alters a later decision for a class constraining the key positively (In / Exists / Gt / Lt: Compatible with
    // the undefined key fails, with NotIn [v] it may pass) or when the key is a topology key (nodeDomains, Record).
    // Such keys are the mutable keys; a class (relaxation stage) with a NotIn / DoesNotExist requirement on one is a
    // mutator, and a consolidation probe that reschedules a mutator's pod keeps per-node requirement copies
    // (consolidate_kernel's MUT variant).  Without mutators every probe treats node requirements as immutable.
    {
        std::vector<uint8_t> neg(K, 0), pos(K, 0), undef(K, 0), topo(K, 0);
        for (int i = 0; i < C; i++)
            for (auto& kv : creq[i]) {
                const HReq& q = kv.second;
                const bool ng = (q.complement && !q.vals.empty()) || (!q.complement && q.vals.empty());
                (ng ? neg : pos)[kv.first] = 1;
            }
        for (const HGroup& g : th.g) topo[g.key] = 1;
        std::vector<uint8_t> has(K, 0);
        for (int j = 0; j < E; j++) {
            for (auto& kv : exlab[j]) has[kv.first] = 1;
            for (int k = 0; k < K; k++) {
                if (!has[k]) undef[k] = 1;
            }
            for (auto& kv : exlab[j]) has[kv.first] = 0;
        }
        c->cons_mutcls.assign(C, 0);
        for (int i = 0; i < C; i++)
            for (auto& kv : creq[i]) {
                const HReq& q = kv.second;
                const int k = kv.first;
                const bool ng = (q.complement && !q.vals.empty()) || (!q.complement && q.vals.empty());
                if (ng && undef[k] && (pos[k] || topo[k])) c->cons_mutcls[i] = 1;
            }
    }
    // ---- key layout ----
    std::vector<uint32_t> kflags(K, 0);
    std::vector<int32_t> kcat(K, -1), kmulti(K, -1), woff(K), nw(K), nval(K), vbase(K);
    std::vector<uint8_t> isint;
    std::vector<int64_t> ival;
    int DW = 0;
    for (int k = 0; k < K; k++) {
        const KeyDict& kd = c->sol.keys[k];
        if (well_known(kd.name)) kflags[k] |= KF_WELL_KNOWN;
        if (k < c->Kcat && c->cat_kflags[k]) {
            kflags[k] |= c->cat_kflags[k];
            kcat[k] = k;
            kmulti[k] = c->cat_multi[k];
        } else if (k == c->key_resvid && c->resvid_rows) {  // values per type: its ResvTab rows (DoesNotExist: dne_mask)
            kflags[k] |= KF_RESV_ROWS;
            kcat[k] = k;
        }
        nval[k] = (int)kd.vals.size();
        nw[k] = std::max(1, (nval[k] + 63) / 64);
        woff[k] = DW;
        DW += nw[k];
        vbase[k] = (int)isint.size();
        for (auto& s : kd.vals) {
            int64_t x = 0;
            isint.push_back(go_atoi(s.c_str(), x) ? 1 : 0);
            ival.push_back(x);
        }
        if ((kflags[k] & KF_CAT_MULTI) && nval[k] > 64)
            return fail(ctx, KP_E_UNSUPPORTED, "multi-valued label with > 64 values after adding pod values");
    }
    // topology keys the device narrows per value: multi-valued catalog labels (zone, capacity-type, zone-id, ...) and
    // labels no instance type carries, each with at most 64 values; hostname is handled per host
    for (const HGroup& g : th.g) {
        if (g.host) continue;
        if ((kflags[g.key] & KF_CAT_SINGLE) || nval[g.key] > 64)
            return fail(ctx, KP_E_UNSUPPORTED, "topology key " + c->sol.keys[g.key].name +
                                                   ": single-valued instance-type labels or > 64 values are not supported");
    }
    PREP_MARK(1);
    // ---- class digests: pod classes then templates ----
    const int CT = C + NT;
    std::vector<ReqHdr> chdr((size_t)CT * K);
    std::vector<uint64_t> cwords((size_t)CT * DW, 0);
    std::vector<int32_t> koff(CT + 1, 0), ckeys, cwsoff;
    std::vector<uint8_t> ckneu;  // parallel to ckeys: key added for topology narrowing only
    std::vector<uint32_t> cflags(CT, 0);
    std::vector<int32_t> min_keys((size_t)NT * KP_MAX_CLASS_KEYS, -1);
    std::vector<int32_t> xkoff(C + 1, 0), xkeys;
    std::vector<uint8_t> hblock(std::max(C, 1), 0);
    bool mayfix = false;
    auto encode = [&](int row, const std::map<int, HReq>& rq) -> bool {
        int so = 0, nk = 0;
        for (auto& kv : rq) {
            const HReq& q = kv.second;
            ReqHdr h{};
            h.flags = RF_DEF | (q.complement ? RF_CMP : 0u) | (q.has_gt ? RF_GT : 0u) | (q.has_lt ? RF_LT : 0u) |
                      (q.has_min ? RF_MIN : 0u);
            h.minv = q.minv;
            h.gt = q.gt;
            h.lt = q.lt;
            chdr[(size_t)row * K + q.key] = h;
            for (int vv : q.vals) cwords[(size_t)row * DW + woff[q.key] + vv / 64] |= 1ull << (vv % 64);
            if (row < C) {
                xkeys.push_back(q.key);
                if ((q.complement && !q.vals.empty()) || (!q.complement && q.vals.empty())) mayfix = true;  // NotIn / DNE
                if (q.key == hostname_key) {
                    // every new NodeClaim carries hostname In [a fresh placeholder]: only NotIn / Exists (no bounds)
                    // intersect it; the merged value stays the placeholder and is dropped at FinalizeScheduling
                    if (!(q.complement && !q.has_gt && !q.has_lt)) hblock[row] = 1;
                    continue;
                }
            }
            nk++;
            ckeys.push_back(q.key);
            ckneu.push_back(0);
            cwsoff.push_back(so);
            so += nw[q.key];
            if (q.key == c->key_zone || q.key == c->key_ct || q.key == c->key_zoneid || q.key == c->key_resvid ||
                q.key == c->key_resvtype)
                cflags[row] |= CF_OFFERING;
        }
        if (row < C && !th.g.empty()) {
            // keys the class's topology groups narrow (AddRequirements adds zone In [domain] even when the pod does
            // not constrain the zone): carried as Exists, skipped by Compatible, merged as the base requirement
            for (int k : th.neutral[row]) {
                ReqHdr h{};
                h.flags = RF_DEF | RF_CMP;
                chdr[(size_t)row * K + k] = h;
                nk++;
                ckeys.push_back(k);
                ckneu.push_back(1);
                cwsoff.push_back(so);
                so += nw[k];
                if (k == c->key_zone || k == c->key_ct || k == c->key_zoneid || k == c->key_resvid || k == c->key_resvtype)
                    cflags[row] |= CF_OFFERING;
            }
            if (!th.cons[row].empty() || !th.rec[row].empty()) cflags[row] |= CF_TOPO;
            if (!th.cons[row].empty()) cflags[row] |= CF_TOPO_CONS;
            bool qrec = true;
            for (int gi : th.rec[row]) {
                const HGroup& g = th.g[gi];
                // an owner's pods satisfy their own node filter: the group's when the owner's semantics are the first
                // owner's (an owner of the identity with another filter records through the group's, topo_record)
                if (!g.inverse && g.type == KP_TOPO_SPREAD && (g.pol & 1) && !g.same[row]) qrec = false;
            }
            if (qrec) cflags[row] |= CF_TOPO_QREC;
        }
        if (nk == 0) cflags[row] |= CF_NOKEYS;  // no requirement keys: NodeClaim.Add = tolerations + Fits (+ minValues)
        if (nk > KP_MAX_CLASS_KEYS || so > KP_MAX_SCR_WORDS) return false;
        koff[row + 1] = (int)ckeys.size();
        if (row < C) xkoff[row + 1] = (int)xkeys.size();
        return true;
    };
    for (int i = 0; i < C; i++)
        if (!encode(i, creq[i])) return fail(ctx, KP_E_UNSUPPORTED, "pod class constrains too many labels");
    for (int j = 0; j < NT; j++) {
        if (!encode(C + j, treq[j])) return fail(ctx, KP_E_UNSUPPORTED, "NodePool constrains too many labels");
        int q = 0;
        for (auto& kv : treq[j])
            if (kv.second.has_min) {
                min_keys[(size_t)j * KP_MAX_CLASS_KEYS + q++] = kv.first;
                c->any_min_values = true;
                if (kv.first < c->Kcat && (c->cat_kflags[kv.first] & KF_CAT_MULTI)) c->min_multi = true;
            }
    }
    // spread node-filter rows after the templates: each Honor spread group's filter is its owner's rows
    std::vector<int2> frow(C, make_int2(0, 0));
    xkoff.resize(CT + 1, xkoff[C]);  // template rows: no keys
    {
        int F = 0;
        for (int i = 0; i < C; i++) F += (int)cfilt[i].size();
        chdr.resize((size_t)(CT + F) * K);
        cwords.resize((size_t)(CT + F) * DW, 0);
        int row = CT;
        for (int i = 0; i < C; i++) {
            frow[i] = make_int2(row, (int)cfilt[i].size());
            for (auto& rq : cfilt[i]) {
                for (auto& kv : rq) {
                    const HReq& q = kv.second;
                    ReqHdr h{};
                    h.flags = RF_DEF | (q.complement ? RF_CMP : 0u) | (q.has_gt ? RF_GT : 0u) | (q.has_lt ? RF_LT : 0u);
                    h.gt = q.gt;
                    h.lt = q.lt;
                    chdr[(size_t)row * K + q.key] = h;
                    for (int vv : q.vals) cwords[(size_t)row * DW + woff[q.key] + vv / 64] |= 1ull << (vv % 64);
                    xkeys.push_back(q.key);
                }
                xkoff.push_back((int)xkeys.size());
                row++;
            }
        }
    }
    // ---- templates: taints, daemon overhead, limits, instance-type rows ----
    std::vector<uint64_t> tol(std::max(C, 1), 0);
    std::vector<int64_t> daemon((size_t)NT * R, 0), remaining((size_t)NT * R, 0);
    std::vector<uint8_t> limit_set((size_t)NT * R, 0);
    std::vector<uint64_t> rows((size_t)NT * TW, 0);
    c->tmpl_np.assign(npo.begin(), npo.end());
    for (int j = 0; j < NT; j++) {
        const kp_nodepool& np = in->nodepools[npo[j]];
        for (int i = 0; i < C; i++) {
            bool all = true;
            for (int q = 0; q < np.n_taints && all; q++)
                all = tolerates(np.taints[q], in->classes[i].tolerations, in->classes[i].n_tolerations);
            if (all) tol[i] |= 1ull << j;
        }
        for (int r = 0; r < R; r++) {
            if (np.daemon_overhead) daemon[(size_t)j * R + r] = np.daemon_overhead[r];
            if (np.limit_set && np.limit_set[r]) {
                limit_set[(size_t)j * R + r] = 1;
                remaining[(size_t)j * R + r] = np.limit_remaining[r];
            }
        }
        if (np.n_types < 0) {
            for (int t = 0; t < T; t++) rows[(size_t)j * TW + t / 64] |= 1ull << (t % 64);
        } else {
            for (int q = 0; q < np.n_types; q++) {
                const int t = np.type_index[q];
                if (t < 0 || t >= T) return fail(ctx, KP_E_INVALID, "nodepool type_index out of range");
                rows[(size_t)j * TW + t / 64] |= 1ull << (t % 64);
            }
        }
    }
    for (int i = 0; i < C; i++)
        if (hblock[i]) tol[i] = 0;  // hostname requirement no new or in-flight NodeClaim can satisfy
    // ---- existing nodes: digests, tolerations ----
    const int EW = (E + 63) / 64;
    std::vector<ReqHdr> exhdr((size_t)std::max(E, 1) * K);
    memset(exhdr.data(), 0, exhdr.size() * sizeof(ReqHdr));
    std::vector<uint64_t> exw((size_t)std::max(E, 1) * DW, 0), extol((size_t)std::max(C, 1) * std::max(EW, 1), 0);
    std::vector<int64_t> exav((size_t)std::max(E, 1) * R, 0), exrq((size_t)std::max(E, 1) * R, 0);
    for (int j = 0; j < E; j++) {
        const kp_existing_node& en = in->existing[j];
        for (auto& kv : exlab[j]) {
            ReqHdr& h = exhdr[(size_t)j * K + kv.first];
            h.flags = RF_DEF;
            exw[(size_t)j * DW + woff[kv.first] + kv.second / 64] |= 1ull << (kv.second % 64);
        }
        for (int r = 0; r < R; r++) {
            exav[(size_t)j * R + r] = en.available[r];
            exrq[(size_t)j * R + r] = en.requests ? en.requests[r] : 0;
        }
        for (int i = 0; i < C; i++) {
            bool all = true;
            for (int q = 0; q < en.n_taints && all; q++)
                all = tolerates(en.taints[q], in->classes[i].tolerations, in->classes[i].n_tolerations);
            if (all) extol[(size_t)i * EW + j / 64] |= 1ull << (j % 64);
        }
    }
    PREP_MARK(2);
    // ---- pods ----
    // per-pod arrays: pinned ctx buffers kept across calls (no allocation or page faults per solve, DMA uploads); the
    // previous solve's uploads from them have finished before they are rewritten
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(c->p_pcls.ensure(std::max(P, 1)));
    HIPCHK(c->p_pshape.ensure(std::max(P, 1)));
    HIPCHK(c->p_preq.ensure((size_t)std::max(P, 1) * R));
    HIPCHK(c->p_fields.ensure((size_t)std::max(P, 1) * 4));
    int32_t* const pcls = c->p_pcls.p;
    int32_t* const pshape = c->p_pshape.p;
    int64_t* const preq = c->p_preq.p;
    int64_t* const fields = c->p_fields.p;
    int cpu_axis = -1, mem_axis = -1;
    for (int r = 0; r < R; r++) {
        if (c->resource_names[r] == "cpu") cpu_axis = r;
        if (c->resource_names[r] == "memory") mem_axis = r;
    }
    if (cpu_axis < 0 || mem_axis < 0) return fail(ctx, KP_E_INVALID, "catalog lacks cpu/memory axes");
    std::vector<uint8_t> active(R, 0);
    for (int j = 0; j < NT; j++)
        for (int r = 0; r < R; r++)
            if (daemon[(size_t)j * R + r] != 0) active[r] = 1;
    // shapes: (class, requests) interned in an open-addressing table of shape ids; a shape's requests point at the
    // pinned row of its first pod (relaxation stages share the row of the shape they relax)
    struct ShapeRec {
        int cls;
        const int64_t* req;
    };
    std::vector<ShapeRec> shapes;
    std::vector<int32_t>& stab = c->h_shape_tab;
    size_t SHT = 1024;
    while (SHT < (size_t)P * 2) SHT <<= 1;
    if (stab.size() < SHT) stab.resize(SHT);
    std::fill(stab.begin(), stab.begin() + SHT, -1);
    auto shape_hash = [&](int cl, const int64_t* rq) {
        uint64_t h = (uint64_t)(uint32_t)cl * 0x9E3779B97F4A7C15ull;
        for (int r = 0; r < R; r++) h = (h ^ (uint64_t)rq[r]) * 0xBF58476D1CE4E5B9ull + 0x94D049BB133111EBull;
        return (size_t)(h ^ (h >> 31));
    };
    auto shape_id = [&](int cl, const int64_t* rq) -> int {
        if (shapes.size() * 2 >= SHT) {  // keep the load ≤ 1/2 (relaxation stages can add shapes beyond P)
            SHT <<= 1;
            stab.assign(SHT, -1);
            for (size_t i = 0; i < shapes.size(); i++) {
                size_t h = shape_hash(shapes[i].cls, shapes[i].req) & (SHT - 1);
                while (stab[h] >= 0) h = (h + 1) & (SHT - 1);
                stab[h] = (int32_t)i;
            }
        }
        for (size_t h = shape_hash(cl, rq) & (SHT - 1);; h = (h + 1) & (SHT - 1)) {
            const int id = stab[h];
            if (id < 0) {
                stab[h] = (int32_t)shapes.size();
                shapes.push_back({cl, rq});
                return (int)shapes.size() - 1;
            }
            if (shapes[id].cls == cl && memcmp(shapes[id].req, rq, sizeof(int64_t) * R) == 0) return id;
        }
    };
    // NewQueue's UID tie-break enters as the UID's first 8 bytes; distinct UIDs sharing them are detected with an
    // open-addressing table over those prefixes (ctx scratch, cleared per call)
    size_t HT = 1024;
    while (HT < (size_t)P * 2) HT <<= 1;
    std::vector<uint64_t>& uid_k = c->h_uid_k;
    std::vector<int32_t>& uid_p = c->h_uid_p;
    if (uid_k.size() < HT) {
        uid_k.resize(HT);
        uid_p.resize(HT);
    }
    std::fill(uid_p.begin(), uid_p.begin() + HT, -1);
    bool uid_collision = false;
    const kp_pods_view& pv = in->pods;
    // kp_pods_view.uids is optional (NULL, or NULL entries): a missing UID is the empty string
    auto uid_of = [&](int p) -> const char* { return pv.uids && pv.uids[p] ? pv.uids[p] : ""; };
    // two independent passes over the pods, run side by side on the ctx's worker pool for large batches: the rows
    // (class, requests, shapes) and the NewQueue keys (the UID strings are separate host allocations, a pointer chase)
    const char* perr = nullptr;
    auto pod_rows = [&]() {
        int prev_shape = -1;
        for (int p = 0; p < P; p++) {
            const int cl = pv.class_id[p];
            if (cl < 0 || cl >= C) {
                perr = "pod class out of range";
                return;
            }
            pcls[p] = cl;
            const int64_t* rq = pv.requests + (size_t)p * R;
            int64_t* dst = &preq[(size_t)p * R];
            for (int r = 0; r < R; r++) {
                dst[r] = rq[r];
                if (rq[r] != 0) active[r] = 1;
                if (rq[r] < 0) {
                    perr = "negative request";
                    return;
                }
            }
            // shapes are numbered in order of first appearance; a pod with the previous pod's class and requests (the
            // pods of one Deployment, typically) reuses its shape without a lookup
            if (p > 0 && cl == pcls[p - 1] && memcmp(dst, dst - R, sizeof(int64_t) * R) == 0) {
                pshape[p] = prev_shape;
            } else {
                pshape[p] = prev_shape = shape_id(cl, dst);
            }
        }
    };
    auto pod_keys = [&]() {
        for (int p = 0; p < P; p++) {
            // NewQueue key: cpu desc, memory desc, creation asc, UID asc.  The UID enters as its first 8 bytes
            // (big-endian, order-preserving); if two distinct UIDs share that prefix, exact string ranks are used.
            if (pv.uids && p + 16 < P && pv.uids[p + 16]) __builtin_prefetch(pv.uids[p + 16]);
            const char* u = uid_of(p);
            uint64_t uk = 0;
            const char* q = u;
            for (int i = 0; i < 8; i++) {
                uk <<= 8;
                if (*q) uk |= (uint8_t)*q++;
            }
            const int64_t* rq = pv.requests + (size_t)p * R;
            fields[(size_t)p * 4 + 0] = rq[cpu_axis];
            fields[(size_t)p * 4 + 1] = rq[mem_axis];
            fields[(size_t)p * 4 + 2] = pv.creation_ns ? pv.creation_ns[p] : 0;
            fields[(size_t)p * 4 + 3] = (int64_t)(uk ^ 0x8000000000000000ull);
            if (!uid_collision) {
                size_t h = (size_t)((uk * 0x9E3779B97F4A7C15ull) >> 20) & (HT - 1);
                for (;; h = (h + 1) & (HT - 1)) {
                    if (uid_p[h] < 0) {
                        uid_k[h] = uk;
                        uid_p[h] = p;
                        break;
                    }
                    if (uid_k[h] == uk) {
                        if (strcmp(uid_of(uid_p[h]), u) != 0) uid_collision = true;
                        break;
                    }
                }
            }
        }
    };
    // KPSIM_PREP_SPLIT_MIN: the batch size from which the two passes run side by side (tests force small batches)
    static const int split_min = getenv("KPSIM_PREP_SPLIT_MIN") ? atoi(getenv("KPSIM_PREP_SPLIT_MIN")) : 16384;
    if (P >= split_min) {
        c->pool.grow(2);
        if (!c->pool.run(2, [&](int t) { t == 0 ? pod_rows() : pod_keys(); }))
            return fail(ctx, KP_E_INVALID, "kp_solve_prepare: host error in a worker thread");
    } else {
        pod_rows();
        pod_keys();
    }
    if (perr) return fail(ctx, KP_E_INVALID, perr);
    if (uid_collision) {
        std::vector<int> idx(P);
        for (int p = 0; p < P; p++) idx[p] = p;
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return strcmp(uid_of(a), uid_of(b)) < 0; });
        int rank = 0;
        for (int i = 0; i < P; i++) {
            if (i > 0 && strcmp(uid_of(idx[i]), uid_of(idx[i - 1])) != 0) rank = i;
            fields[(size_t)idx[i] * 4 + 3] = (int64_t)((uint64_t)rank ^ 0x8000000000000000ull);
        }
    }
    PREP_MARK(3);
    // relaxation stages of every shape: shape_next[s] = the shape of (relax_next[class of s], the same requests)
    std::vector<int32_t> shape_next;
    if (!c->pref.relax_next.empty()) {
        for (size_t sid = 0; sid < shapes.size(); sid++) {
            const int nx = c->pref.relax_next[shapes[sid].cls];
            shape_next.push_back(nx >= 0 ? shape_id(nx, shapes[sid].req) : -1);
        }
    }
    KpDev& d = c->dev;
    d = KpDev{};
    d.n_active = 0;
    for (int r = 0; r < R; r++)
        if (active[r]) d.active_axes[d.n_active++] = r;
    PREP_MARK(4);
    // ---- device buffers ----
    hipStream_t s = c->stream;
    std::vector<ReqHdr> empty_hdr(K);
    memset(empty_hdr.data(), 0, empty_hdr.size() * sizeof(ReqHdr));
    std::vector<uint64_t> empty_words(DW, 0);
    HIPCHK(c->d_kflags.upload(kflags, s));
    HIPCHK(c->d_kcat.upload(kcat, s));
    HIPCHK(c->d_kmulti.upload(kmulti, s));
    HIPCHK(c->d_woff.upload(woff, s));
    HIPCHK(c->d_nw.upload(nw, s));
    HIPCHK(c->d_nval.upload(nval, s));
    HIPCHK(c->d_vbase.upload(vbase, s));
    if (isint.empty()) {
        isint.push_back(0);
        ival.push_back(0);
    }
    HIPCHK(c->d_val_isint.upload(isint, s));
    HIPCHK(c->d_val_int.upload(ival, s));
    HIPCHK(c->d_cls_koff.upload(koff, s));
    if (ckeys.empty()) {
        ckeys.push_back(0);
        cwsoff.push_back(0);
        ckneu.push_back(0);
    }
    HIPCHK(c->d_cls_kneutral.upload(ckneu, s));
    HIPCHK(c->d_cls_keys.upload(ckeys, s));
    HIPCHK(c->d_cls_wsoff.upload(cwsoff, s));
    HIPCHK(c->d_cls_hdr.upload(chdr, s));
    HIPCHK(c->d_cls_words.upload(cwords, s));
    HIPCHK(c->d_cls_flags.upload(cflags, s));
    HIPCHK(c->d_V.ensure((size_t)CT * TW));
    HIPCHK(c->d_tmpl_rows.upload(rows, s));
    HIPCHK(c->d_tmpl_opts.ensure((size_t)std::max(NT, 1) * TW));
    HIPCHK(c->d_tmpl_ok.ensure(std::max(NT, 1)));
    HIPCHK(c->d_tol.upload(tol, s));
    HIPCHK(c->d_daemon.upload(daemon, s));
    HIPCHK(c->d_limit_set.upload(limit_set, s));
    HIPCHK(c->d_remaining.upload(remaining, s));
    c->h_remaining = remaining;
    HIPCHK(c->d_min_keys.upload(min_keys, s));
    if (xkeys.empty()) xkeys.push_back(0);
    HIPCHK(c->d_cls_xkoff.upload(xkoff, s));
    HIPCHK(c->d_cls_xkeys.upload(xkeys, s));
    HIPCHK(c->d_ex_hdr0.upload(exhdr, s));
    HIPCHK(c->d_ex_words0.upload(exw, s));
    HIPCHK(c->d_ex_hdr.ensure(exhdr.size()));
    HIPCHK(c->d_ex_words.ensure(exw.size()));
    HIPCHK(c->d_ex_avail.upload(exav, s));
    HIPCHK(c->d_ex_req.upload(exrq, s));
    HIPCHK(c->d_ex_head.ensure((size_t)KP_MAX_R * std::max(E, 1)));
    HIPCHK(c->d_ex_static.ensure(std::max(E, 1)));
    HIPCHK(c->d_ex_tol.upload(extol, s));
    HIPCHK(c->d_XT.ensure(extol.size()));
    HIPCHK(c->d_pod_cls.upload(pcls, P, s));
    HIPCHK(c->d_pod_shape.upload(pshape, P, s));
    if (!shape_next.empty()) {
        HIPCHK(c->d_pod_cls0.upload(pcls, P, s));
        HIPCHK(c->d_pod_shape0.upload(pshape, P, s));
        HIPCHK(c->d_relax_next.upload(c->pref.relax_next, s));
        HIPCHK(c->d_shape_next.upload(shape_next, s));
        HIPCHK(c->d_last_ep.ensure(std::max(P, 1)));
    }
    HIPCHK(c->d_pod_req.upload(preq, (size_t)P * R, s));
    HIPCHK(c->d_sort_fields.upload(fields, (size_t)P * 4, s));
    HIPCHK(c->d_empty_hdr.upload(empty_hdr, s));
    HIPCHK(c->d_empty_words.upload(empty_words, s));
    // in-flight NodeClaim capacity.  A self-selecting hostname anti-affinity (required, or preferred under Respect: each
    // pod takes a new NodeClaim before anything is relaxed) puts every pod of its class on a host of its own, a
    // self-selecting hostname spread at most maxSkew per host: when that lower bound exceeds the first plan
    // (KP_NC_FIRST), the solve is planned for it from the start, so a node-dense Deployment runs one execute.  A solve
    // that still overflows (kp_solve_fetch) makes the next prepare of this ctx, and only that one, plan for every pod.
    int64_t dense = 0;  // a lower bound of the NodeClaims: the largest such class, less the existing nodes
    {
        std::vector<int64_t> ccount(std::max(C, 1), 0);
        for (int p = 0; p < P; p++) ccount[in->pods.class_id[p]]++;
        for (const HGroup& g : th.g)
            if (!g.inverse && g.host) {
                int64_t m = 0;  // pods of the self-selecting classes that own the group
                for (int o = 0; o < C; o++)
                    if (g.memb[o] && g.sel[o]) m += ccount[o];
                int64_t n = 0;
                if (g.type == KP_TOPO_ANTI_AFFINITY) n = m;
                else if (g.type == KP_TOPO_SPREAD && g.skew > 0) n = (m + g.skew - 1) / g.skew;
                dense = std::max(dense, n - E);
            }
    }
    int64_t plan = c->nc_cap_once > 0 ? c->nc_cap_once : KP_NC_FIRST;
    c->nc_cap_once = 0;
    if (dense + dense / 8 + 64 > plan) plan = dense + dense / 8 + 64;
    const int NCcap = (int)std::min<int64_t>(std::min<int64_t>(plan, KP_MAX_NC), std::max(P, 1));
    c->last_plan_nc = NCcap;
    HIPCHK(c->d_nc_hdr.ensure((size_t)NCcap * K));
    HIPCHK(c->d_nc_words.ensure((size_t)NCcap * DW));
    HIPCHK(c->d_nc_opts.ensure((size_t)NCcap * TW));
    HIPCHK(c->d_nc_req.ensure((size_t)NCcap * R));
    HIPCHK(c->d_nc_tmpl.ensure(NCcap));
    HIPCHK(c->d_nc_held.ensure((size_t)NCcap * std::max(1, c->h_ro.ridw)));
    HIPCHK(c->d_nc_rlive.ensure(NCcap));
    HIPCHK(c->d_qbuf.ensure(std::max(P, 1)));
    HIPCHK(c->d_last_len.ensure(std::max(P, 1)));
    HIPCHK(c->d_pod_result.ensure(std::max(P, 1)));
    HIPCHK(c->d_pod_order.ensure(std::max(P, 1)));
    HIPCHK(c->d_perm_a.ensure(std::max(P, 1)));
    HIPCHK(c->d_perm_b.ensure(std::max(P, 1)));
    HIPCHK(c->d_keys_a.ensure(std::max(P, 1)));
    HIPCHK(c->d_keys_b.ensure(std::max(P, 1)));
    HIPCHK(c->d_nc_count.ensure(1));
    HIPCHK(c->d_err.ensure(1));
    HIPCHK(c->d_nc_npods.ensure(NCcap));
    HIPCHK(c->d_nc_slice_pos.ensure(NCcap));
    HIPCHK(c->d_nc_nopts.ensure(NCcap));
    HIPCHK(c->d_nc_valid.ensure(NCcap));
    HIPCHK(c->d_nc_ntypes.ensure(NCcap));
    const int M = in->max_instance_types > 0 ? std::min(in->max_instance_types, T) : T;
    HIPCHK(c->d_nc_types.ensure((size_t)NCcap * M));
    HIPCHK(c->d_stats.ensure(ST_COUNT));
    // ---- topology: groups, initial domains (buildDomainGroups), per-class group lists, tie-break ranks ----
    const int G = (int)th.g.size();
    c->tg_G = G;
    c->tg_HG = th.n_host;
    c->tg_host_aff.assign(std::max(G, 1), 0);
    for (int gi = 0; gi < G; gi++)
        c->tg_host_aff[gi] = th.g[gi].host && th.g[gi].type == KP_TOPO_AFFINITY && !th.g[gi].inverse;
    c->cons_dec.assign(c->cons_extra_ncand, {});
    c->cons_hdec.assign(c->cons_extra_ncand, {});
    c->cons_hlost.assign(c->cons_extra_ncand, {});
    c->h_tpos0.clear();
    {
        const int G1 = std::max(G, 1);
        std::vector<int4> tinfo(G1);
        std::vector<int32_t> thr_row(G1, -1), towner(G1, 0), tpol(G1, 0), tcnt0((size_t)G1 * 64, 0), tpos0(G1, 0);
        std::vector<int2> tfrow(G1, make_int2(0, 0));
        std::vector<int32_t> tlate(G1, -1);
        std::vector<uint64_t> tknown0(G1, 0);
        std::vector<int32_t> tcoff(C + 1, 0), tcl, troff(C + 1, 0), trl;
        std::vector<KpTopoCons> tce;
        std::vector<int2> tce_hosts;  // KpTopoCons.hdom lists
        std::vector<int> tce_hosts_g; // ... the entry's group
        std::vector<KpTopoRec> tre;
        std::vector<uint8_t> vrank((size_t)K * 64, 0xFF);
        // hostname rows: existing nodes, then NodeClaim ids 0 .. NCcap, the last a spare that stays 0 (a template
        // evaluation for a NodeClaim at capacity reads it; the capacity check then reports the overflow)
        const int HN = E + NCcap + 1;
        std::vector<int32_t> hc0((size_t)std::max(1, th.n_host) * HN, 0);
        if (G > 0) {
            auto hreq_has = [&](const HReq& q, int v) {
                const bool in = std::binary_search(q.vals.begin(), q.vals.end(), v);
                if (!q.complement) return in;
                if (in) return false;
                if (!q.has_gt && !q.has_lt) return true;
                int64_t x = 0;
                if (!go_atoi(c->sol.keys[q.key].vals[v].c_str(), x)) return false;
                return !((q.has_gt && q.gt >= x) || (q.has_lt && q.lt <= x));
            };
            // buildDomainGroups: value → the NodePools (templates) offering it, over every NodePool × its types
            std::map<int, std::map<int, std::vector<int>>> dg;
            auto domains_of = [&](int k) -> const std::map<int, std::vector<int>>& {
                auto it = dg.find(k);
                if (it != dg.end()) return it->second;
                std::map<int, std::vector<int>>& m = dg[k];
                const int mi = k < c->Kcat ? c->cat_multi[k] : -1;
                for (int j = 0; j < NT; j++) {
                    auto npit = treq[j].find(k);
                    const bool hp = npit != treq[j].end();
                    for (int t = 0; t < T; t++) {
                        if (!((rows[(size_t)j * TW + t / 64] >> (t % 64)) & 1ull)) continue;
                        const int st = mi >= 0 ? c->h_multi_state[(size_t)mi * T + t] : KP_LABEL_ABSENT;
                        const bool ht = st != KP_LABEL_ABSENT;
                        if (!hp && !ht) continue;
                        const uint64_t tm = st == KP_LABEL_IN ? c->h_multi_mask[(size_t)mi * T + t] : 0ull;
                        if (hp && ht) {
                            for (uint64_t x = tm; x; x &= x - 1) {
                                const int v = __builtin_ctzll(x);
                                if (hreq_has(npit->second, v)) m[v].push_back(j);
                            }
                        } else if (hp) {
                            for (int v : npit->second.vals) m[v].push_back(j);  // requirement.Values()
                        } else {
                            for (uint64_t x = tm; x; x &= x - 1) m[__builtin_ctzll(x)].push_back(j);
                        }
                    }
                    if (hp && !npit->second.complement && !npit->second.vals.empty())  // NodePool In requirements
                        for (int v : npit->second.vals) m[v].push_back(j);
                }
                return m;
            };
            auto owner_tolerates = [&](int owner, int j) {
                const kp_nodepool& np = in->nodepools[npo[j]];
                for (int q = 0; q < np.n_taints; q++)
                    if (!tolerates(np.taints[q], in->classes[owner].tolerations, in->classes[owner].n_tolerations)) return false;
                return true;
            };
            for (int gi = 0; gi < G; gi++) {
                const HGroup& g = th.g[gi];
                tinfo[gi] = make_int4(g.type | (g.inverse ? TG_INVERSE : 0) | (g.host ? TG_HOST : 0), g.key, g.skew, g.mindom);
                thr_row[gi] = g.hrow;
                towner[gi] = g.owner;
                tpol[gi] = g.pol;
                if (!g.inverse && g.type == KP_TOPO_SPREAD && (g.pol & 1)) tfrow[gi] = frow[g.owner];
                tlate[gi] = th.g_late[gi];
                if (g.host) continue;
                for (auto& kv : domains_of(g.key)) {
                    bool ok = !(g.type == KP_TOPO_SPREAD && (g.pol & 2));
                    for (size_t q = 0; q < kv.second.size() && !ok; q++) ok = owner_tolerates(g.owner, kv.second[q]);
                    if (ok) tknown0[gi] |= 1ull << kv.first;
                }
                // value ranks by name (the canonical pick among equal counts)
                const auto& vals = c->sol.keys[g.key].vals;
                std::vector<int> idx(vals.size());
                for (size_t v = 0; v < vals.size(); v++) idx[v] = (int)v;
                std::sort(idx.begin(), idx.end(), [&](int a, int b) { return vals[a] < vals[b]; });
                for (size_t r = 0; r < idx.size(); r++) vrank[(size_t)g.key * 64 + idx[r]] = (uint8_t)r;
            }
            for (int i = 0; i < C; i++) {
                for (int e : th.cons[i]) tcl.push_back(e);
                for (int e : th.rec[i]) trl.push_back(e);
                tcoff[i + 1] = (int)tcl.size();
                troff[i + 1] = (int)trl.size();
            }
            // the entries' static operands (KpTopoCons / KpTopoRec): req_has over the encoded class digest, as the device
            // evaluates it
            auto digest_has = [&](int row, int k, int v) {
                const ReqHdr& h = chdr[(size_t)row * K + k];
                const bool bit = (cwords[(size_t)row * DW + woff[k] + v / 64] >> (v % 64)) & 1ull;
                bool within = true;
                if (h.flags & (RF_GT | RF_LT)) {
                    const int b = vbase[k] + v;
                    within = isint[b] && !((h.flags & RF_GT) && h.gt >= ival[b]) && !((h.flags & RF_LT) && h.lt <= ival[b]);
                }
                return (h.flags & RF_CMP) ? (!bit && within) : (bit && within);
            };
            for (int i = 0; i < C; i++) {
                for (int e : th.cons[i]) {
                    const int gi = e & 0x3FFFFFFF, self = (e >> 30) & 1;
                    const HGroup& g = th.g[gi];
                    KpTopoCons t{};
                    t.g = gi;
                    t.flags = g.type | (self << 2) | (g.host ? 8 : 0);
                    t.skew = g.skew;
                    t.mindom = g.mindom;
                    if (g.host) {
                        t.key = -1 - g.hrow;
                        // nextDomainAffinity counts the positive domains podDomains admits: a pod requiring the hostname
                        // (In / NotIn a list; Exists admits every host) lists the existing nodes its values name
                        const auto& rq = c->pref.has_strict[i] ? cstrict[i] : creq[i];
                        const auto hit = rq.find(g.key);
                        if (g.type == KP_TOPO_AFFINITY && self && !g.inverse && hit != rq.end()) {
                            const HReq& q = hit->second;
                            if (!(q.complement && q.vals.empty() && !q.has_gt && !q.has_lt)) {
                                const int off = (int)tce_hosts.size();
                                if (!q.has_gt && !q.has_lt)  // bounds admit no host name (Has parses an integer)
                                    for (int v : q.vals) {
                                        const auto f = host_node.find(v);
                                        if (f == host_node.end()) continue;
                                        tce_hosts.push_back(make_int2(f->second, 0));
                                        tce_hosts_g.push_back(gi);
                                    }
                                t.hdom = (((int)tce_hosts.size() - off) << 2) | (q.complement ? 2 : 1);
                                t.podhas = (uint64_t)off;
                            }
                        }
                    } else {
                        t.key = g.key;
                        // podDomains: the strict requirements' (no preferred term) requirement for the key, else Exists
                        const bool strict = c->pref.has_strict[i] != 0;
                        const auto sit = strict ? cstrict[i].find(g.key) : cstrict[i].end();
                        for (int v = 0; v < 64 && v < nval[g.key]; v++) {
                            t.vmask |= 1ull << v;
                            const bool has = strict ? (sit == cstrict[i].end() || hreq_has(sit->second, v)) : digest_has(i, g.key, v);
                            if (has) t.podhas |= 1ull << v;
                        }
                    }
                    tce.push_back(t);
                }
                for (int gi : th.rec[i]) {
                    const HGroup& g = th.g[gi];
                    KpTopoRec r{};
                    r.g = gi;
                    r.flags = g.type | (g.inverse ? 4 : 0) | (g.host ? 8 : 0);
                    r.key = g.host ? -1 - g.hrow : g.key;
                    r.late = th.g_late[gi];
                    if (!g.inverse && g.type == KP_TOPO_SPREAD && (g.pol & 2))
                        for (int j = 0; j < NT; j++)
                            if (!((tol[g.owner] >> j) & 1ull)) r.skip |= 1ull << j;
                    tre.push_back(r);
                }
            }
            // countDomains over the pods bound to existing nodes (forward groups that select the pod's class; a spread
            // group's node filter against the node's labels and taints) and updateInverseAffinities (the inverse
            // anti-affinity groups of the bound pod's class record the node's domain) — [core] scheduling/topology.go,
            // restated in oracle/orc_solve.cpp build_topology.  A node without the key's label is not counted.
            auto node_val = [&](int j, int k) {
                for (auto& e : exlab[j])
                    if (e.first == k) return e.second;
                return -1;
            };
            // TopologyNodeFilter.MatchesRequirements: Compatible(node labels, a filter row of the owner), no wk allowance
            auto node_compatible_with = [&](int j, int owner) {
                for (auto& rq : cfilt[owner]) {
                    bool ok = true;
                    for (auto& kv : rq) {
                        const HReq& q = kv.second;
                        const int v = node_val(j, kv.first);
                        const bool qno = (q.complement && !q.vals.empty()) || (!q.complement && q.vals.empty());
                        if (v < 0) {
                            if (!qno) ok = false;
                        } else if (!hreq_has(q, v)) {
                            ok = false;
                        }
                        if (!ok) break;
                    }
                    if (ok) return true;
                }
                return false;
            };
            auto node_tolerated_by = [&](int j, int owner) {
                const kp_existing_node& en = in->existing[j];
                for (int q = 0; q < en.n_taints; q++)
                    if (!tolerates(en.taints[q], in->classes[owner].tolerations, in->classes[owner].n_tolerations)) return false;
                return true;
            };
            c->h_tknown_dg.assign(tknown0.begin(), tknown0.end());  // buildDomainGroups only (consolidation probes)
            // one bound pod of class b on node j; cand >= 0: a consolidation candidate's reschedulable pod, whose
            // value-keyed contributions are also kept per candidate (a probe takes off the pods it reschedules)
            auto count_pod = [&](int j, int b, int cand) -> bool {
                for (int gi = 0; gi < G; gi++) {
                    const HGroup& g = th.g[gi];
                    if (g.inverse ? !g.memb[b] : !g.sel[b]) continue;
                    if (!g.inverse && g.type == KP_TOPO_SPREAD) {
                        if ((g.pol & 1) && !node_compatible_with(j, g.owner)) continue;
                        if ((g.pol & 2) && !node_tolerated_by(j, g.owner)) continue;
                    }
                    if (g.host) {
                        if (hc0[(size_t)g.hrow * HN + j]++ == 0) tpos0[gi]++;
                        if (cand >= 0 && c->tg_host_aff[gi]) c->cons_hdec[cand][gi]++;
                    } else {
                        const int v = node_val(j, g.key);
                        if (v < 0) continue;
                        if (v >= 64) return false;
                        tcnt0[(size_t)gi * 64 + v]++;
                        tknown0[gi] |= 1ull << v;
                        if (cand >= 0) {
                            auto& row = c->cons_dec[cand][gi];
                            if (row.empty()) row.assign(64, 0);
                            row[v]++;
                        }
                    }
                }
                return true;
            };
            for (int i = 0; i < in->n_bound; i++) {
                const int j = in->bound_node[i], b = in->bound_class[i];
                if (j < 0 || j >= E || b < 0 || b >= C) return fail(ctx, KP_E_INVALID, "bound pod index out of range");
                if (!count_pod(j, b, -1)) return fail(ctx, KP_E_UNSUPPORTED, "topology key with more than 64 values");
            }
            // kp_consolidate_prepare: each candidate's reschedulable pods are bound to its node in the cluster
            c->cons_dec.assign(c->cons_extra_ncand, {});
            c->cons_hdec.assign(c->cons_extra_ncand, {});
            c->cons_hlost.assign(c->cons_extra_ncand, {});
            std::vector<int> cand_node(c->cons_extra_ncand, -1);
            for (auto& e : c->cons_extra) {
                if (!count_pod(e[0], in->pods.class_id[e[1]], e[2]))
                    return fail(ctx, KP_E_UNSUPPORTED, "topology key with more than 64 values");
                cand_node[e[2]] = e[0];
            }
            for (int ci = 0; ci < c->cons_extra_ncand; ci++)
                for (auto& kv : c->cons_hdec[ci])
                    if (hc0[(size_t)th.g[kv.first].hrow * HN + cand_node[ci]] == kv.second) c->cons_hlost[ci].push_back(kv.first);
            // hostname lists (KpTopoCons.hdom): a candidate's node keeps a selected pod its probe does not reschedule
            std::map<int, int> node_cand;
            for (int ci = 0; ci < c->cons_extra_ncand; ci++) node_cand[cand_node[ci]] = ci;
            for (size_t q = 0; q < tce_hosts.size(); q++) {
                const int j = tce_hosts[q].x, gi = tce_hosts_g[q];
                int left = hc0[(size_t)th.g[gi].hrow * HN + j];
                const auto nc = node_cand.find(j);
                if (nc != node_cand.end()) {
                    const auto dec = c->cons_hdec[nc->second].find(gi);
                    if (dec != c->cons_hdec[nc->second].end()) left -= dec->second;
                }
                tce_hosts[q].y = left > 0;
            }
            c->h_tpos0.assign(tpos0.begin(), tpos0.end());
        }
        if (tcl.empty()) tcl.push_back(0);
        if (trl.empty()) trl.push_back(0);
        if (tce.empty()) tce.push_back(KpTopoCons{});
        if (tce_hosts.empty()) tce_hosts.push_back(make_int2(0, 0));
        HIPCHK(c->d_tce_hosts.upload(tce_hosts, s));
        if (tre.empty()) tre.push_back(KpTopoRec{});
        HIPCHK(c->d_cls_tce.upload(tce, s));
        HIPCHK(c->d_cls_tre.upload(tre, s));
        HIPCHK(c->d_tg_info.upload(tinfo, s));
        HIPCHK(c->d_tg_hrow.upload(thr_row, s));
        HIPCHK(c->d_tg_owner.upload(towner, s));
        HIPCHK(c->d_tg_pol.upload(tpol, s));
        HIPCHK(c->d_tg_frow.upload(tfrow, s));
        // late identities (topo_build): born at the start when a pod of the Solve (its input class) owns them
        // TopoSnap rows the FFD kernel's LDS plan holds: the most constraining groups of any class (at most KP_SNAP_ROWS)
        d.snap_rows = 1;
        for (int i = 0; i < C && G > 0; i++)
            d.snap_rows = std::max(d.snap_rows, std::min((int)th.cons[i].size(), (int)KP_SNAP_ROWS));
        c->tg_nlate = G > 0 ? th.n_late : 0;
        c->h_cls_birth.assign(std::max(C, 1), 0);
        d.born0 = 0;
        if (c->tg_nlate > 0) {
            HIPCHK(c->d_tg_late.upload(tlate, s));
            c->h_cls_birth.assign(th.cls_birth.begin(), th.cls_birth.end());
            HIPCHK(c->d_cls_birth.upload(c->h_cls_birth, s));
            // NewTopology over the pods in input order: a variant is born only while no sibling is (topo_birth)
            for (int i = 0; i < P; i++) d.born0 = late_birth(th.late_sib, d.born0, th.cls_birth[in->pods.class_id[i]]);
        }
        c->tg_var = c->tg_nlate > 0 && th.any_var;
        c->h_late_sib = th.late_sib;
        if (c->tg_var) {
            HIPCHK(c->d_late_sib.upload(th.late_sib, s));
            HIPCHK(c->d_late_grp.upload(th.late_grp, s));
        }
        HIPCHK(c->d_tg_cnt0.upload(tcnt0, s));
        HIPCHK(c->d_tg_cnt.ensure(tcnt0.size()));
        HIPCHK(c->d_tg_known0.upload(tknown0, s));
        HIPCHK(c->d_tg_known.ensure(tknown0.size()));
        HIPCHK(c->d_tg_pos0.upload(tpos0, s));
        HIPCHK(c->d_tg_pos.ensure(tpos0.size()));
        HIPCHK(c->d_tg_hcnt0.upload(hc0, s));
        HIPCHK(c->d_tg_hcnt.ensure(hc0.size()));
        HIPCHK(c->d_cls_tcoff.upload(tcoff, s));
        HIPCHK(c->d_cls_tc.upload(tcl, s));
        HIPCHK(c->d_cls_troff.upload(troff, s));
        HIPCHK(c->d_cls_tr.upload(trl, s));
        HIPCHK(c->d_vrank.upload(vrank, s));
        d.HN = HN;
    }
    if (P > 0) {
        size_t tb = 0;
        HIPCHK(kp_queue_sort(nullptr, P, c->d_perm_a.p, c->d_perm_b.p, c->d_keys_a.p, c->d_keys_b.p, nullptr, &tb, s, nullptr));
        HIPCHK(c->d_sort_temp.ensure(tb));
        c->sort_temp_bytes = tb;
    }
    // ---- KpDev ----
    d.T = T;
    d.TW = TW;
    d.R = R;
    d.K = K;
    d.n_slots = c->n_slots;
    d.n_multi = c->n_multi;
    d.type_val = c->d_type_val.p;
    d.multi_mask = c->d_multi_mask.p;
    d.multi16 = c->multi16_ok ? c->d_multi16.p : nullptr;
    d.dne_mask = c->d_dne_mask.p;
    d.alloc = c->d_alloc.p;
    d.cap = c->d_cap.p;
    d.avail_zc = c->d_avail_zc.p;
    d.slot_price = c->d_slot_price.p;
    d.slot_zone = c->d_slot_zone.p;
    d.slot_ct = c->d_slot_ct.p;
    d.slot_zoneid = c->d_slot_zoneid.p;
    d.name_rank = c->d_name_rank.p;
    d.nonneg = c->d_nonneg.p;
    d.kflags = c->d_kflags.p;
    d.kcat = c->d_kcat.p;
    d.kmulti = c->d_kmulti.p;
    d.woff = c->d_woff.p;
    d.nw = c->d_nw.p;
    d.nval = c->d_nval.p;
    d.vbase = c->d_vbase.p;
    d.val_isint = c->d_val_isint.p;
    d.val_int = c->d_val_int.p;
    d.DW = DW;
    d.key_zone = c->key_zone;
    d.key_ct = c->key_ct;
    d.key_zoneid = c->key_zoneid;
    d.key_resvid = c->key_resvid;
    d.key_resvtype = c->key_resvtype;
    d.C = C;
    d.NT = NT;
    d.cls_koff = c->d_cls_koff.p;
    d.cls_keys = c->d_cls_keys.p;
    d.cls_wsoff = c->d_cls_wsoff.p;
    d.cls_hdr = c->d_cls_hdr.p;
    d.cls_words = c->d_cls_words.p;
    d.cls_flags = c->d_cls_flags.p;
    d.V = c->d_V.p;
    d.tmpl_rows = c->d_tmpl_rows.p;
    d.tmpl_opts = c->d_tmpl_opts.p;
    d.tmpl_ok = c->d_tmpl_ok.p;
    d.tol = c->d_tol.p;
    d.daemon = c->d_daemon.p;
    d.limit_set = c->d_limit_set.p;
    d.remaining = c->d_remaining.p;
    HIPCHK(c->d_tmpl_lmask.ensure((size_t)std::max(1, d.NT) * std::max(1, d.TW)));
    d.tmpl_lmask = c->d_tmpl_lmask.p;
    d.min_keys = c->d_min_keys.p;
    d.E = E;
    d.EW = EW;
    d.ex_hdr0 = c->d_ex_hdr0.p;
    d.ex_words0 = c->d_ex_words0.p;
    d.ex_hdr = c->d_ex_hdr.p;
    d.ex_words = c->d_ex_words.p;
    d.ex_avail = c->d_ex_avail.p;
    d.ex_req = c->d_ex_req.p;
    d.ex_head = c->d_ex_head.p;
    d.ex_static = c->d_ex_static.p;
    d.XT = c->d_XT.p;
    d.ex_tol = c->d_ex_tol.p;
    d.cls_xkoff = c->d_cls_xkoff.p;
    d.cls_xkeys = c->d_cls_xkeys.p;
    d.ex_mayfix = mayfix ? 1 : 0;
    d.P = P;
    d.pod_cls = c->d_pod_cls.p;
    d.pod_shape = c->d_pod_shape.p;
    const bool relax = !c->pref.relax_next.empty();
    d.relax_next = relax ? c->d_relax_next.p : nullptr;
    d.shape_next = relax ? c->d_shape_next.p : nullptr;
    d.pod_cls0 = relax ? c->d_pod_cls0.p : nullptr;
    d.pod_shape0 = relax ? c->d_pod_shape0.p : nullptr;
    d.last_ep = relax ? c->d_last_ep.p : nullptr;
    d.best_effort = c->best_effort ? 1 : 0;
    d.pod_req = c->d_pod_req.p;
    d.queue0 = nullptr;  // set by execute (sort output)
    d.NCcap = NCcap;
    d.nc_hdr = c->d_nc_hdr.p;
    d.nc_words = c->d_nc_words.p;
    d.nc_opts = c->d_nc_opts.p;
    d.nc_req = c->d_nc_req.p;
    d.nc_tmpl = c->d_nc_tmpl.p;
    d.empty_hdr = c->d_empty_hdr.p;
    d.empty_words = c->d_empty_words.p;
    d.qbuf = c->d_qbuf.p;
    d.last_len = c->d_last_len.p;
    d.pod_result = c->d_pod_result.p;
    d.pod_order = c->d_pod_order.p;
    d.nc_count = c->d_nc_count.p;
    d.nc_npods = c->d_nc_npods.p;
    d.nc_slice_pos = c->d_nc_slice_pos.p;
    d.nc_nopts = c->d_nc_nopts.p;
    d.nc_valid = c->d_nc_valid.p;
    d.M = M;
    d.nc_types = c->d_nc_types.p;
    d.nc_ntypes = c->d_nc_ntypes.p;
    d.stats = c->d_stats.p;
    d.err = c->d_err.p;
    d.profile = getenv("KPSIM_PROFILE") ? 1 : 0;
    // topology pods: candidates per block round (KPSIM_TOPO_CANDS, diagnostics)
    {  // topology solves run the KP_NWAVES_TOPO-wave instantiations
        const int nw = G > 0 ? KP_NWAVES_TOPO : KP_NWAVES;
        d.topo_cands = getenv("KPSIM_TOPO_CANDS") ? std::max(1, std::min(nw, atoi(getenv("KPSIM_TOPO_CANDS")))) : nw;
    }
    d.team_eval = getenv("KPSIM_NO_TEAM") ? 0 : 1;  // diagnostics: KPSIM_NO_TEAM=1 evaluates topology candidates one per wave
    d.noop_quick = getenv("KPSIM_NO_NOOP") ? 0 : 1;  // diagnostics: KPSIM_NO_NOOP=1 disables the no-op merge quick accept
    d.team_first = getenv("KPSIM_NO_TEAM_FIRST") ? 0 : 1;  // diagnostics: KPSIM_NO_TEAM_FIRST=1 evaluates it beside the others
    d.block_sort = getenv("KPSIM_NO_BLOCK_SORT") ? 0 : 1;  // diagnostics: KPSIM_NO_BLOCK_SORT=1 leaves it to wave 0
    // KPSIM_TRACE_POD=p traces pod p; KPSIM_TRACE_CLASS=c traces every slow-path pod of class c (trace_pod = -2 - c)
    d.trace_pod = getenv("KPSIM_TRACE_POD") ? atoi(getenv("KPSIM_TRACE_POD"))
                  : getenv("KPSIM_TRACE_CLASS") ? -2 - atoi(getenv("KPSIM_TRACE_CLASS")) : -1;
    d.trace_max = getenv("KPSIM_TRACE_MAXPOD") ? atoi(getenv("KPSIM_TRACE_MAXPOD")) : INT32_MAX;
    d.trace = nullptr;
    if (d.trace_pod != -1) {
        HIPCHK(c->d_trace.ensure(1 + 6 * KP_TRACE_N + 3 + 2 * 4096));
        d.trace = c->d_trace.p;
    }
    d.G = G;
    d.key_host = th.key_host;
    d.tg_info = c->d_tg_info.p;
    d.tg_hrow = c->d_tg_hrow.p;
    d.tg_owner = c->d_tg_owner.p;
    d.tg_pol = c->d_tg_pol.p;
    d.tg_frow = c->d_tg_frow.p;
    d.tg_late = c->tg_nlate > 0 ? c->d_tg_late.p : nullptr;
    d.cls_birth = c->tg_nlate > 0 ? c->d_cls_birth.p : nullptr;
    d.late_sib = c->tg_var ? c->d_late_sib.p : nullptr;
    d.late_grp = c->tg_var ? c->d_late_grp.p : nullptr;
    d.tg_cnt = c->d_tg_cnt.p;
    d.tg_known = c->d_tg_known.p;
    d.tg_hcnt = c->d_tg_hcnt.p;
    d.tg_pos = c->d_tg_pos.p;
    d.cls_tcoff = c->d_cls_tcoff.p;
    d.cls_tc = c->d_cls_tc.p;
    d.cls_troff = c->d_cls_troff.p;
    d.cls_tr = c->d_cls_tr.p;
    d.cls_tce = c->d_cls_tce.p;
    d.tce_hosts = c->d_tce_hosts.p;
    d.cls_tre = c->d_cls_tre.p;
    d.cls_kneutral = c->d_cls_kneutral.p;
    d.vrank = c->d_vrank.p;
    // quick-accept headroom scale per active axis: every allocatable value >> qshift fits in 30 bits
    for (int ai = 0; ai < KP_LDS_AXES; ai++) {
        int sh = 0;
        if (ai < d.n_active) {
            int64_t mx = 0;
            for (int t = 0; t < T; t++) mx = std::max(mx, c->alloc_rt[(size_t)d.active_axes[ai] * T + t]);
            while ((mx >> sh) > 0x3FFFFFFF) sh++;
        }
        d.qshift[ai] = sh;
    }
    d.ro = c->h_ro.n > 0 ? c->d_ro.p : nullptr;
    d.type_ro = c->d_type_ro.p;
    d.ro_price = c->d_ro_price.p;
    d.ro_n = c->h_ro.n;
    d.ro_w = c->h_ro.w;
    d.ro_nrid = c->h_ro.nrid;
    d.ro_ridw = c->h_ro.ridw;
    d.resv_on = (c->reserved_capacity && c->h_ro.n > 0) ? 1 : 0;
    d.rcap0 = c->d_rcap0.p;
    d.nc_held = c->d_nc_held.p;
    d.nc_rlive = c->d_nc_rlive.p;
    d.alloc_act = nullptr;
    if (NCcap > KP_NC_FIRST || T > 1024) {  // node-dense plan or large catalog: the staged axes' allocatable table in HBM
                                            // ([axes][TP], TP = 64-padded T) when LDS cannot hold it
        const int TP = (T + 63) / 64 * 64, ns = std::min(d.n_active, KP_LDS_AXES);
        std::vector<int64_t> act((size_t)std::max(ns, 1) * TP, 0);
        for (int ai = 0; ai < ns; ai++)
            for (int t = 0; t < T; t++) act[(size_t)ai * TP + t] = c->alloc_rt[(size_t)d.active_axes[ai] * T + t];
        HIPCHK(c->d_alloc_stage.upload(act, s));
        d.alloc_act = c->d_alloc_stage.p;
        // HBM slice arrays, used when the plan holds more NodeClaims than LDS (kp_ffd_plan_lds)
        HIPCHK(c->d_g_key.ensure(NCcap));
        HIPCHK(c->d_g_ord.ensure(NCcap));
        HIPCHK(c->d_g_last.ensure(NCcap));
        HIPCHK(c->d_g_tmpl.ensure(NCcap));
        d.g_key = c->d_g_key.p;
        d.g_ord = c->d_g_ord.p;
        d.g_last = c->d_g_last.p;
        d.g_tmpl = c->d_g_tmpl.p;
    }
    if (!kp_ffd_plan_lds(d, KP_LDS_BYTES)) return fail(ctx, KP_E_UNSUPPORTED, "FFD kernel LDS plan exceeds 160 KB");
    if (getenv("KPSIM_PROFILE"))
        fprintf(stderr, "[kpsim] FFD LDS plan: fixed block %zu B, quick rows %d (axes %d), NodeClaim slots %d, allocatable %s, "
                "%d B of %d\n", d.G > 0 ? kp_ffd_shared_bytes_topo() : kp_ffd_shared_bytes(), d.lds_nq, d.lds_A, d.lds_ncmax, d.alloc_global ? "HBM" : "LDS",
                d.lds_bytes, KP_LDS_BYTES);
    c->P = P;
    c->C = C;
    c->NT = NT;
    c->K = K;
    c->DW = DW;
    c->M = M;
    HIPCHK(hipStreamSynchronize(s));
    c->ns_prep = ns_since(t0);
    c->prepared = true;
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

// ---------------------------------------------------------------------------------------------
// solve: execute (device only)
// ---------------------------------------------------------------------------------------------
extern "C" kp_status kp_solve_execute(kp_ctx* ctx) {
    if (!ctx) return KP_E_INVALID;
    ctx->cons_prep_valid = false;
    ctx->cons_gen++;  // cached pass rows and read-backs of kp_consolidate_command are stale
    if (!ctx->prepared || !ctx->have_catalog) return fail(ctx, KP_E_STATE, "kp_solve_execute before kp_solve_prepare");
    HIPCHK(hipSetDevice(ctx->device));
    kp_ctx* c = ctx;
    KpDev& d = c->dev;
    hipStream_t s = c->stream;
    const auto t0 = clk::now();
    // per-call state (remaining limits are mutated by the FFD kernel)
    HIPCHK(hipMemsetAsync(c->d_nc_count.p, 0, sizeof(int32_t), s));
    HIPCHK(hipMemsetAsync(c->d_err.p, 0, sizeof(int32_t), s));
    if (!c->h_remaining.empty())
        HIPCHK(hipMemcpyAsync(c->d_remaining.p, c->h_remaining.data(), c->h_remaining.size() * sizeof(int64_t),
                              hipMemcpyHostToDevice, s));
    if (c->tg_G > 0) {  // topology counts start from the bound pods' counts (TopologyGroup state per Solve)
        HIPCHK(hipMemcpyAsync(c->d_tg_cnt.p, c->d_tg_cnt0.p, (size_t)c->tg_G * 64 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_tg_known.p, c->d_tg_known0.p, (size_t)c->tg_G * 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_tg_pos.p, c->d_tg_pos0.p, (size_t)c->tg_G * 4, hipMemcpyDeviceToDevice, s));
        if (c->tg_HG > 0)
            HIPCHK(hipMemcpyAsync(c->d_tg_hcnt.p, c->d_tg_hcnt0.p, (size_t)c->tg_HG * d.HN * 4, hipMemcpyDeviceToDevice, s));
    }
    int32_t* q0 = nullptr;
    HIPCHK(hipEventRecord(c->ev[0], s));
    if (d.P > 0) {
        size_t tb = c->sort_temp_bytes;
        HIPCHK(kp_queue_sort(c->d_sort_fields.p, d.P, c->d_perm_a.p, c->d_perm_b.p, c->d_keys_a.p, c->d_keys_b.p,
                             c->d_sort_temp.p, &tb, s, &q0));
    }
    d.queue0 = q0;
    if (d.trace) HIPCHK(hipMemsetAsync(d.trace, 0, sizeof(int32_t), s));
    HIPCHK(hipEventRecord(c->ev[1], s));
    HIPCHK(kp_launch_class_mask(d, s));
    HIPCHK(hipEventRecord(c->ev[2], s));
    HIPCHK(kp_launch_template_init(d, s));
    HIPCHK(kp_launch_existing(d, s));
    HIPCHK(c->d_self.ensure(1));
    d.self = c->d_self.p;
    HIPCHK(hipMemcpyAsync(c->d_self.p, &d, sizeof(KpDev), hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(c->ev[3], s));
    HIPCHK(kp_launch_ffd(d, s));
    HIPCHK(hipEventRecord(c->ev[4], s));
    HIPCHK(kp_launch_finalize(d, d.NCcap, s));
    HIPCHK(hipEventRecord(c->ev[5], s));
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < 5; i++) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]));
        c->kernel_ms[i] = ms;
    }
    if (d.trace) {  // KPSIM_TRACE_POD diagnostics
        std::vector<int32_t> tr(1 + 6 * KP_TRACE_N + 3 + 2 * 4096);
        HIPCHK(hipMemcpy(tr.data(), d.trace, tr.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
        fprintf(stderr, "[kpsim trace] pod %d: %d evaluations\n", d.trace_pod, tr[0]);
        for (int i = std::max(0, tr[0] - KP_TRACE_N); i < tr[0]; i++) {  // ring: the last KP_TRACE_N entries
            const int32_t* e = &tr[1 + 6 * (i % KP_TRACE_N)];
            fprintf(stderr, "[kpsim trace]   pod %d nc %d ok %d flags %d pos %d held %08x\n", e[0], e[1], e[2], e[3],
                    e[4], (unsigned)e[5]);
        }
        const int32_t* sl = &tr[1 + 6 * KP_TRACE_N];
        fprintf(stderr, "[kpsim trace] slice N %d scan_start %d first candidate pos %d\n", sl[0], sl[1], sl[2]);
        for (int i = 0; i < std::min(sl[0], 4096); i++)
            fprintf(stderr, "[kpsim trace]   pos %d nc %d pods %d rej %d\n", i, sl[3 + 2 * i], sl[4 + 2 * i] & 0x7FFFFFFF,
                    (int)(((uint32_t)sl[4 + 2 * i]) >> 31));
    }
    c->ns_exec = ns_since(t0);
    c->executed = true;
    return KP_OK;
}

// ---------------------------------------------------------------------------------------------
// solve: fetch (D2H + decode)
// ---------------------------------------------------------------------------------------------
extern "C" kp_status kp_solve_fetch(kp_ctx* ctx, kp_solve_output* out) {
    if (!ctx || !out) return KP_E_INVALID;
    if (!ctx->executed) return fail(ctx, KP_E_STATE, "kp_solve_fetch before kp_solve_execute");
    HIPCHK(hipSetDevice(ctx->device));
    kp_ctx* c = ctx;
    hipStream_t s = c->stream;
    const auto t0 = clk::now();
    int32_t N = 0, err = 0;
    int64_t st[ST_COUNT];
    HIPCHK(hipMemcpyAsync(&N, c->d_nc_count.p, sizeof N, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&err, c->d_err.p, sizeof err, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(st, c->d_stats.p, sizeof st, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    c->nc_overflow = err == 1;
    if (err == 1) {
        c->nc_cap_once = std::min(KP_MAX_NC, std::max(c->P, 1));  // the next prepare plans for every pod, once
        return fail(ctx, KP_E_UNSUPPORTED, "in-flight NodeClaim capacity exceeded");
    }
    if (err) return fail(ctx, KP_E_STATE, "device solve loop exceeded its pop bound (internal error)");
    const int P = c->P, M = c->M;
    std::vector<int32_t> npods(N), spos(N), nopts(N), valid(N), ntypes(N), tmpl(N), types((size_t)N * M), pres(P), pord(P);
    if (N > 0) {
        HIPCHK(hipMemcpyAsync(npods.data(), c->d_nc_npods.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(spos.data(), c->d_nc_slice_pos.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(nopts.data(), c->d_nc_nopts.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(valid.data(), c->d_nc_valid.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(ntypes.data(), c->d_nc_ntypes.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(tmpl.data(), c->d_nc_tmpl.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(types.data(), c->d_nc_types.p, (size_t)N * M * 4, hipMemcpyDeviceToHost, s));
    }
    if (P > 0) {
        HIPCHK(hipMemcpyAsync(pres.data(), c->d_pod_result.p, P * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(pord.data(), c->d_pod_order.p, P * 4, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    c->last_N = N;
    c->h_nc_tmpl = tmpl;
    int n_ids = 0;
    for (int i = 0; i < N; i++) n_ids += ntypes[i];
    out->n_nodeclaims = N;
    out->n_type_ids = n_ids;
    kp_solve_stats& so = out->stats;
    so = kp_solve_stats{};
    so.pods_popped = st[ST_POPPED];
    so.nodeclaim_evals = st[ST_NC_EVALS];
    so.nodeclaim_candidates_scanned = st[ST_NC_SCANNED];
    so.template_evals = st[ST_TMPL_EVALS];
    so.existing_evals = st[ST_EXIST_PLACED];
    so.sorts_fast = st[ST_SORT_FAST];
    so.sorts_full = st[ST_SORT_FULL];
    for (int i = 0; i < 6; i++) c->cycles[i] = st[ST_CYC_POP + i];
    for (int i = 0; i < 6; i++) c->cycles[6 + i] = st[ST_EV_REQ + i];
    for (int i = 0; i < 7; i++) c->cycles[12 + i] = st[ST_QUICK + i];
    for (int i = 0; i < 11; i++) c->cycles[19 + i] = st[ST_N_NOINV + i];
    for (int i = 0; i < 3; i++) c->cycles[30 + i] = st[ST_TOPO_QUICK + i];
    for (int i = 0; i < 4; i++) c->cycles[33 + i] = st[ST_REJ_REQ + i];
    if (getenv("KPSIM_PROFILE") && st[ST_SLOW_WHY] + st[ST_SLOW_WHY + 1] + st[ST_SLOW_WHY + 2] + st[ST_SLOW_WHY + 3])
        fprintf(stderr, "[kpsim] slow-path pods: no candidate %lld, class not absorbed %lld, witness short %lld, no witness table %lld; "
                "no-op merge quick accepts %lld; placed by the first candidate %lld, a later one %lld, the templates %lld; "
                "block-evaluated first candidates %lld; cycles: commit + templates %lld, class cache fills %lld\n",
                (long long)st[ST_SLOW_WHY], (long long)st[ST_SLOW_WHY + 1], (long long)st[ST_SLOW_WHY + 2],
                (long long)st[ST_SLOW_WHY + 3], (long long)st[ST_SLOW_WHY + 4], (long long)st[ST_SLOW_WHY + 5],
                (long long)st[ST_SLOW_WHY + 6], (long long)st[ST_SLOW_WHY + 7], (long long)st[ST_SLOW_WHY + 8],
                (long long)st[ST_SLOW_WHY + 9], (long long)st[ST_SLOW_WHY + 10]);
    if (getenv("KPSIM_PROFILE") && st[ST_TQ_WHY] + st[ST_TQ_WHY + 1] + st[ST_TQ_WHY + 2] + st[ST_TQ_WHY + 3] + st[ST_TQ_WHY + 4])
        fprintf(stderr, "[kpsim] topology pods past the prefilter: no survivor %lld, not QREC %lld, no quick row %lld, class not "
                        "absorbed %lld, quick row %lld (witness fits %lld, merge no-op %lld); NQ %d of %d NodeClaims\n",
                (long long)st[ST_TQ_WHY], (long long)st[ST_TQ_WHY + 1], (long long)st[ST_TQ_WHY + 2], (long long)st[ST_TQ_WHY + 3],
                (long long)st[ST_TQ_WHY + 4], (long long)st[ST_TQ_WHY + 5], (long long)st[ST_TQ_WHY + 6], c->dev.lds_nq, N);
    if (getenv("KPSIM_PROFILE") && st[ST_SEG])
        fprintf(stderr, "[kpsim] solve loop segments (cycles): fast loop + slow-path entry %lld, topology section %lld "
                        "(topology quick accepts: %lld iterations, %lld cycles from the slow-path entry), class cache %lld, "
                        "evaluations %lld, commit / templates / slice move %lld\n",
                (long long)st[ST_SEG], (long long)st[ST_SEG + 1], (long long)st[ST_TQ_ITERS], (long long)st[ST_TQ_CYC],
                (long long)st[ST_SEG + 2], (long long)st[ST_SEG + 3], (long long)st[ST_SEG + 4]);
    so.ns_host_prep = c->ns_prep;
    so.ns_device_solve = c->ns_exec;
    if (N > out->cap_nodeclaims || n_ids > out->cap_type_ids) return fail(ctx, KP_E_BUFFER, "output buffers too small");
    int off = 0;
    for (int i = 0; i < N; i++) {
        out->nodeclaim_nodepool[i] = valid[i] ? c->tmpl_np[tmpl[i]] : -1;
        out->nodeclaim_n_pods[i] = npods[i];
        if (out->nodeclaim_slice_pos) out->nodeclaim_slice_pos[i] = spos[i];
        if (out->nodeclaim_n_options) out->nodeclaim_n_options[i] = nopts[i];
        out->nodeclaim_type_offset[i] = off;
        for (int q = 0; q < ntypes[i]; q++) out->type_ids[off++] = types[(size_t)i * M + q];
    }
    out->nodeclaim_type_offset[N] = off;
    for (int p = 0; p < P; p++) {
        int r = pres[p];
        int o = pord[p];
        if (r >= 0 && !valid[r]) {
            r = KP_POD_UNSCHEDULABLE;
            o = -1;
        }
        out->pod_result[p] = r;
        if (out->pod_order) out->pod_order[p] = o;
    }
    so.ns_device_finalize = ns_since(t0);
    so.ns_total = c->ns_prep + c->ns_exec + so.ns_device_finalize;
    return KP_OK;
}

extern "C" kp_status kp_last_kernel_times(kp_ctx* ctx, double* ms, int32_t n) {
    if (!ctx || !ms) return KP_E_INVALID;
    if (!ctx->executed) return fail(ctx, KP_E_STATE, "no execute yet");
    for (int i = 0; i < n && i < 5; i++) ms[i] = ctx->kernel_ms[i];
    for (int i = 5; i < n && i < 42; i++) ms[i] = (double)ctx->cycles[i - 5];
    return KP_OK;
}

extern "C" kp_status kp_solve(kp_ctx* ctx, const kp_solve_input* in, kp_solve_output* out) {
    for (int attempt = 0;; attempt++) {
        kp_status st = kp_solve_prepare(ctx, in);
        if (st != KP_OK) return st;
        st = kp_solve_execute(ctx);
        if (st != KP_OK) return st;
        st = kp_solve_fetch(ctx, out);
        // more in-flight NodeClaims than the plan holds (the prepare's node-dense estimate missed): one more run planned
        // for every pod (kp_solve_fetch set it up for the next prepare only; later solves start from the first plan)
        const int want = std::min(KP_MAX_NC, std::max(in->pods.n_pods, 1));
        if (st == KP_E_UNSUPPORTED && ctx->nc_overflow && attempt == 0 && ctx->last_plan_nc < want) continue;
        ctx->nc_cap_once = 0;
        return st;
    }
}

static std::string reqs_text(const kp_ctx* ctx, const ReqHdr* h, const uint64_t* w);

extern "C" kp_status kp_result_nodeclaim_requirements(kp_ctx* ctx, int32_t nc, char* buf, int64_t cap, int64_t* needed) {
    if (!ctx) return KP_E_INVALID;
    if (!ctx->executed) return fail(ctx, KP_E_STATE, "no solve result");
    if (nc < 0 || nc >= ctx->last_N) return fail(ctx, KP_E_INVALID, "nodeclaim index");
    HIPCHK(hipSetDevice(ctx->device));
    const int K = ctx->K, DW = ctx->DW;
    std::vector<ReqHdr> h(K);
    std::vector<uint64_t> w(DW);
    HIPCHK(hipMemcpy(h.data(), ctx->d_nc_hdr.p + (size_t)nc * K, K * sizeof(ReqHdr), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(w.data(), ctx->d_nc_words.p + (size_t)nc * DW, DW * sizeof(uint64_t), hipMemcpyDeviceToHost));
    const std::string s = reqs_text(ctx, h.data(), w.data());
    if (needed) *needed = (int64_t)s.size() + 1;
    if ((int64_t)s.size() + 1 > cap || !buf) return KP_E_BUFFER;
    memcpy(buf, s.c_str(), s.size() + 1);
    return KP_OK;
}

// A requirements digest (one ReqHdr per solve key, value bitsets at the keys' word offsets) as the text of
// kp_result_nodeclaim_requirements: "key \t complement \t gt \t lt \t minValues \t sorted values" lines, sorted.
static std::string reqs_text(const kp_ctx* ctx, const ReqHdr* h, const uint64_t* w) {
    const int K = ctx->K;
    std::vector<std::string> lines;
    int off = 0;
    for (int k = 0; k < K; k++) {
        const KeyDict& kd = ctx->sol.keys[k];
        const int nwk = std::max(1, ((int)kd.vals.size() + 63) / 64);
        const int wo = off;
        off += nwk;
        if (!(h[k].flags & RF_DEF)) continue;
        std::string l = kd.name + "\t" + ((h[k].flags & RF_CMP) ? "1" : "0") + "\t" +
                        ((h[k].flags & RF_GT) ? std::to_string(h[k].gt) : "-") + "\t" +
                        ((h[k].flags & RF_LT) ? std::to_string(h[k].lt) : "-") + "\t" +
                        ((h[k].flags & RF_MIN) ? std::to_string(h[k].minv) : "-") + "\t";
        std::vector<std::string> vs;
        for (int v = 0; v < (int)kd.vals.size(); v++)
            if ((w[wo + v / 64] >> (v % 64)) & 1ull) vs.push_back(kd.vals[v]);
        std::sort(vs.begin(), vs.end());
        for (size_t i = 0; i < vs.size(); i++) {
            if (i) l += '\x1f';
            l += vs[i];
        }
        lines.push_back(l);
    }
    std::sort(lines.begin(), lines.end());
    std::string s;
    for (auto& l : lines) s += l + "\n";
    return s;
}

// ---------------------------------------------------------------------------------------------
// consolidation probes (kp_consolidate): encode the cluster with kp_solve_prepare, then one wave per probe
// ---------------------------------------------------------------------------------------------
extern "C" int32_t kp_consolidate_probe_count(const kp_consolidate_input* in) {
    if (!in) return 0;
    const int n = in->n_candidates;
    const int ns = n > 0 ? n : 0;
    const int mx = in->max_candidates > 0 ? in->max_candidates : 100;
    const int nm = n < 2 ? 0 : (n <= mx ? n - 1 : mx);  // firstNConsolidationOption: mid in [1, max], candidates[0 : mid+1]
    if (in->mode == KP_CONSOLIDATE_SINGLE) return ns;
    if (in->mode == KP_CONSOLIDATE_MULTI) return nm;
    return nm + ns;  // KP_CONSOLIDATE_BOTH
}

static kp_status cons_prepare_one(kp_ctx* ctx, const kp_consolidate_input* in) try {
    if (!ctx || !in) return KP_E_INVALID;
    ctx->cons_prepared = false;
    ctx->cons_prep_valid = false;
    ctx->cons_gen++;  // cached pass rows and read-backs of kp_consolidate_command are stale
    if (ctx->has_reserved && !ctx->ro_ok)
        return fail(ctx, KP_E_UNSUPPORTED, "consolidation over this catalog: " + ctx->ro_why);
    if (!ctx->solve_unsupported.empty()) return fail(ctx, KP_E_UNSUPPORTED, "consolidation: " + ctx->solve_unsupported);
    if (in->mode != KP_CONSOLIDATE_SINGLE && in->mode != KP_CONSOLIDATE_MULTI)
        return fail(ctx, KP_E_INVALID, "unknown consolidation mode");
    const kp_solve_input& cl = in->cluster;
    const int P = cl.pods.n_pods, E = cl.n_existing, NC = in->n_candidates;
    // inputs: candidates on distinct nodes, each pod pending or owned by one candidate, prices >= 0
    {
        std::vector<uint8_t> seen_pod(std::max(P, 1), 0), seen_node(std::max(E, 1), 0);
        for (int i = 0; i < in->n_pending; i++) {
            const int p = in->pending[i];
            if (p < 0 || p >= P || seen_pod[p]++) return fail(ctx, KP_E_INVALID, "pending pod out of range or repeated");
        }
        for (int ci = 0; ci < NC; ci++) {
            const kp_candidate& cd = in->candidates[ci];
            if (cd.node < 0 || cd.node >= E || seen_node[cd.node]++) return fail(ctx, KP_E_INVALID, "candidate node out of range or repeated");
            if (!(cd.price >= 0) || cd.price > DBL_MAX) return fail(ctx, KP_E_INVALID, "candidate price must be finite and >= 0");
            if (cd.n_pods < 0 || (cd.n_pods > 0 && !cd.pods)) return fail(ctx, KP_E_INVALID, "candidate pods");
            for (int i = 0; i < cd.n_pods; i++) {
                const int p = cd.pods[i];
                if (p < 0 || p >= P || seen_pod[p]++) return fail(ctx, KP_E_INVALID, "candidate pod out of range or repeated");
            }
        }
    }
    // topology: every candidate's reschedulable pods are bound to its node in the cluster (base counts); kp_solve_prepare
    // also keeps each candidate's value-keyed contributions (cons_dec) so that a probe takes off the pods it reschedules
    ctx->cons_extra.clear();
    ctx->cons_extra_ncand = NC;
    for (int ci = 0; ci < NC; ci++)
        for (int q = 0; q < in->candidates[ci].n_pods; q++)
            ctx->cons_extra.push_back({in->candidates[ci].node, in->candidates[ci].pods[q], ci});
    ctx->cons_pend.assign(in->pending, in->pending + in->n_pending);
    ctx->cons_topo = true;
    kp_status st = kp_solve_prepare(ctx, &cl);
    ctx->cons_topo = false;
    ctx->cons_pend.clear();
    ctx->cons_extra.clear();
    ctx->cons_extra_ncand = 0;
    if (st != KP_OK) return st;
    kp_ctx* c = ctx;
    // preference relaxation (PREFERENCE_POLICY=Respect), MIN_VALUES_POLICY=BestEffort, hostname pod affinity and minValues
    // on multi-valued labels run inside the probes as in the Solve (consolidate_kernel: relaxed queue entries, the Add's
    // relaxed minValues, per-probe positive hostname domains, prefix-OR distinct counts)
    const KpDev& d = c->dev;
    if (d.M <= 0 || d.M > 64) return fail(ctx, KP_E_UNSUPPORTED, "consolidation needs max_instance_types in 1..64");
    const int T = c->T, TW = c->TW, R = c->R, A = d.n_active;
    hipStream_t s = c->stream;
    KpCons& k = c->cons;
    k = KpCons{};
    k.n_cand = NC;
    k.spot_to_spot = in->spot_to_spot ? 1 : 0;
    c->cons_max_candidates = in->max_candidates > 0 ? in->max_candidates : 100;
    c->cons_n_pending = in->n_pending;
    k.v_spot = k.v_od = -1;
    if (c->key_ct >= 0) {
        k.v_spot = c->sol.keys[c->key_ct].find("spot");
        k.v_od = c->sol.keys[c->key_ct].find("on-demand");
    }
    for (int sl = 0; sl < c->n_slots; sl++) {
        if (c->slot_ct[sl] == k.v_spot && k.v_spot >= 0) k.spot_slots |= 1ull << sl;
        if (c->slot_ct[sl] == k.v_od && k.v_od >= 0) k.od_slots |= 1ull << sl;
    }
    std::vector<int> np_tmpl(cl.n_nodepools, -1);
    for (int j = 0; j < (int)c->tmpl_np.size(); j++) np_tmpl[c->tmpl_np[j]] = j;
    std::vector<int32_t> ci((size_t)std::max(NC, 1) * 4, 0), cpods;
    std::vector<int32_t>& coff = c->cons_off;
    coff.assign(NC + 1, 0);
    std::vector<double> cprice(std::max(NC, 1), 0.0);
    std::vector<int64_t> ccap((size_t)std::max(NC, 1) * R, 0);
    for (int i = 0; i < NC; i++) {
        const kp_candidate& cd = in->candidates[i];
        ci[i * 4 + 0] = cd.node;
        ci[i * 4 + 1] = cd.capacity_type;
        ci[i * 4 + 2] = cd.instance_type >= 0 && cd.instance_type < T ? cd.instance_type : -1;
        ci[i * 4 + 3] = cd.nodepool >= 0 && cd.nodepool < cl.n_nodepools && cd.capacity ? np_tmpl[cd.nodepool] : -1;
        cprice[i] = cd.price;
        if (cd.capacity)
            for (int r = 0; r < R; r++) ccap[(size_t)i * R + r] = cd.capacity[r];
        coff[i + 1] = coff[i] + cd.n_pods;
        for (int q = 0; q < cd.n_pods; q++) cpods.push_back(cd.pods[q]);
    }
    if (cpods.empty()) cpods.push_back(0);
    std::vector<int32_t> pend(in->pending, in->pending + in->n_pending);
    if (pend.empty()) pend.push_back(0);
    std::vector<uint64_t> init(std::max(d.EW, 1), 0);
    for (int j = 0; j < E; j++)
        if (!in->initialized || in->initialized[j]) init[j >> 6] |= 1ull << (j & 63);
    const int astride = TW * 64;
    std::vector<int64_t> act((size_t)std::max(A, 1) * astride, 0);
    for (int ai = 0; ai < A; ai++)
        for (int t = 0; t < T; t++) act[(size_t)ai * astride + t] = c->alloc_rt[(size_t)d.active_axes[ai] * T + t];
    k.PW = std::max(1, (P + 63) / 64);
    k.astride = astride;
    HIPCHK(c->d_cand_i.upload(ci, s));
    HIPCHK(c->d_cand_off.upload(coff, s));
    HIPCHK(c->d_cand_pods.upload(cpods, s));
    HIPCHK(c->d_pending.upload(pend, s));
    HIPCHK(c->d_cand_price.upload(cprice, s));
    HIPCHK(c->d_cand_cap.upload(ccap, s));
    HIPCHK(c->d_init.upload(init, s));
    HIPCHK(c->d_alloc_act.upload(act, s));
    // topology: the starting decrements of every probe — single-node probe ci: candidate ci's rows; multi-node probe i:
    // the sum over candidates [0, i + 2) — one row of 64 value counts per group
    k.G = c->tg_G;
    k.HG = c->tg_HG;
    if (k.G > 0) {
        std::vector<int32_t> soff(NC + 1, 0), dg, dv;
        for (int ci = 0; ci < NC; ci++) {
            for (auto& kv : c->cons_dec[ci]) {
                dg.push_back(kv.first);
                dv.insert(dv.end(), kv.second.begin(), kv.second.end());
            }
            soff[ci + 1] = (int32_t)dg.size();
        }
        const int mx = c->cons_max_candidates;
        const int nm = NC < 2 ? 0 : (NC <= mx ? NC - 1 : mx);
        std::vector<int32_t> moff(nm + 1, (int32_t)dg.size());
        std::map<int, std::vector<int32_t>> acc;
        auto add = [&](int ci) {
            for (auto& kv : c->cons_dec[ci]) {
                auto& row = acc[kv.first];
                if (row.empty()) row.assign(64, 0);
                for (int v = 0; v < 64; v++) row[v] += kv.second[v];
            }
        };
        for (int i = 0; i < nm; i++) {
            if (i == 0) add(0);
            add(i + 1);
            for (auto& kv : acc) {
                dg.push_back(kv.first);
                dv.insert(dv.end(), kv.second.begin(), kv.second.end());
            }
            moff[i + 1] = (int32_t)dg.size();
        }
        if (dg.empty()) {
            dg.push_back(0);
            dv.assign(64, 0);
        }
        HIPCHK(c->d_dec_soff.upload(soff, s));
        HIPCHK(c->d_dec_moff.upload(moff, s));
        HIPCHK(c->d_dec_g.upload(dg, s));
        HIPCHK(c->d_dec_v.upload(dv, s));
        HIPCHK(c->d_pt_dgk.upload(c->h_tknown_dg, s));
        // hostname pod affinity: each probe's positive-domain count per group (the base minus the domains only its
        // candidates' pods held)
        std::vector<int32_t> ha(k.G, -1), hg;
        for (int gi = 0; gi < k.G; gi++)
            if (c->tg_host_aff[gi]) {
                ha[gi] = (int)hg.size();
                hg.push_back(gi);
            }
        k.n_ha = (int)hg.size();
        std::vector<int32_t> hp((size_t)std::max(1, (NC + nm) * k.n_ha), 0);
        if (k.n_ha > 0) {
            std::vector<int32_t> acc(k.n_ha, 0);
            for (int ci = 0; ci < NC; ci++) {
                for (int ga = 0; ga < k.n_ha; ga++) hp[(size_t)ci * k.n_ha + ga] = c->h_tpos0[hg[ga]];
                for (int g : c->cons_hlost[ci]) hp[(size_t)ci * k.n_ha + ha[g]]--;
            }
            for (int i = 0; i < nm; i++) {  // multi-node probe i: candidates [0, i + 2)
                for (int cc = i == 0 ? 0 : i + 1; cc < i + 2; cc++)
                    for (int g : c->cons_hlost[cc]) acc[ha[g]]++;
                for (int ga = 0; ga < k.n_ha; ga++) hp[(size_t)(NC + i) * k.n_ha + ga] = c->h_tpos0[hg[ga]] - acc[ga];
            }
        }
        HIPCHK(c->d_tg_ha.upload(ha, s));
        HIPCHK(c->d_hpos0.upload(hp, s));
    }
    // mutators (kp_solve_prepare): a probe that reschedules a pod whose class, or a relaxation stage of it, may change a
    // node's requirements runs on the MUT variant (per-probe node requirement copies); the others are unaffected
    {
        const int C0 = cl.n_classes;
        std::vector<uint8_t> chain(std::max(C0, 1), 0);
        for (int i = 0; i < C0; i++)
            for (int s = i; s >= 0 && !chain[i]; s = c->pref.relax_next.empty() ? -1 : c->pref.relax_next[s])
                if (s < (int)c->cons_mutcls.size() && c->cons_mutcls[s]) chain[i] = 1;
        auto pod_mut = [&](int p) { return chain[cl.pods.class_id[p]] != 0; };
        bool pend_mut = false;
        for (int i = 0; i < in->n_pending; i++) pend_mut = pend_mut || pod_mut(in->pending[i]);
        const int mx = c->cons_max_candidates;
        const int nm = NC < 2 ? 0 : (NC <= mx ? NC - 1 : mx);
        std::vector<int32_t> ms(std::max(NC, 1), 0), mm(std::max(nm, 1), 0);
        int any = 0, pre = pend_mut ? 1 : 0;
        for (int ci = 0; ci < NC; ci++) {
            int f = pend_mut ? 1 : 0;
            for (int q = 0; q < in->candidates[ci].n_pods && !f; q++) f = pod_mut(in->candidates[ci].pods[q]) ? 1 : 0;
            ms[ci] = f;
            any |= f;
            pre |= f;  // multi-node probe i covers candidates [0, i + 2)
            if (ci >= 1 && ci - 1 < nm) mm[ci - 1] = pre;
        }
        k.mut = any;
        c->cons_n_mut = 0;
        for (int ci = 0; ci < NC; ci++) c->cons_n_mut += ms[ci];
        for (int i = 0; i < nm; i++) c->cons_n_mut += mm[i];
        HIPCHK(c->d_mut_s.upload(ms, s));
        HIPCHK(c->d_mut_m.upload(mm, s));
        // late topology identities a probe's NewTopology creates: owned by its pending pods or its candidates' pods
        k.born_s = k.born_m = nullptr;
        if (c->tg_nlate > 0) {
            // in the probe's pod order (pending, then its candidates' pods): a variant is born only while no sibling
            // is, so each probe starts with its own first owner's variant
            const std::vector<uint64_t>& sib = c->tg_var ? c->h_late_sib : std::vector<uint64_t>();
            uint64_t bp = 0;
            for (int i = 0; i < in->n_pending; i++) bp = late_birth(sib, bp, c->h_cls_birth[cl.pods.class_id[in->pending[i]]]);
            std::vector<uint64_t> bs(std::max(NC, 1), bp), bm(std::max(nm, 1), bp);
            uint64_t acc = bp;
            for (int ci = 0; ci < NC; ci++) {
                for (int q = 0; q < in->candidates[ci].n_pods; q++) {
                    const uint64_t cb = c->h_cls_birth[cl.pods.class_id[in->candidates[ci].pods[q]]];
                    bs[ci] = late_birth(sib, bs[ci], cb);
                    acc = late_birth(sib, acc, cb);
                }
                if (ci >= 1 && ci - 1 < nm) bm[ci - 1] = acc;  // multi-node probe i covers candidates [0, i + 2)
            }
            HIPCHK(c->d_born_s.upload(bs, s));
            HIPCHK(c->d_born_m.upload(bm, s));
            k.born_s = c->d_born_s.p;
            k.born_m = c->d_born_m.p;
        }
    }
    HIPCHK(c->d_next.ensure(3));
    HIPCHK(c->d_rank.ensure(std::max(P, 1)));
    HIPCHK(c->d_pend_bits.ensure(k.PW));
    HIPCHK(c->d_cons_stats.ensure(CS_COUNT));
    HIPCHK(hipStreamSynchronize(s));
    c->cons_prepared = true;
    c->n_pass_launches = c->n_readbacks = 0;
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_consolidate_prepare(kp_ctx* ctx, const kp_consolidate_input* in) try {
    if (!ctx || !in) return KP_E_INVALID;
    return fan_out(ctx, [&](kp_ctx* c) { return cons_prepare_one(c, in); });
} catch (...) {
    return fail(ctx, KP_E_INVALID, "kp_consolidate_prepare: host error");
}

// probes of a prepared pass: multi-node (firstNConsolidationOption's prefixes), single-node, or both (multi first)
static int cons_probes(const kp_ctx* c, int mode) {
    const int NC = c->cons.n_cand;
    const int nm = NC < 2 ? 0 : (NC <= c->cons_max_candidates ? NC - 1 : c->cons_max_candidates);
    return mode == KP_CONSOLIDATE_SINGLE ? NC : mode == KP_CONSOLIDATE_MULTI ? nm : nm + NC;
}

// One device's share of a pass: multi-node probes [m0, m1) and single-node probes [s0, s1) of the prepared pass in one
// launch (the multi-node prefixes first, longest first), results into out_multi[m1 - m0] / out_single[s1 - s0].
// record: kp_consolidate_command's read-back run of one probe (FULL variant only; the replacement NodeClaim lands in
// d_rec_*).
static kp_status cons_run(kp_ctx* ctx, int m0, int m1, int s0, int s1, kp_probe_result* out_multi,
                          kp_probe_result* out_single, bool record = false) try {
    if (!ctx) return KP_E_INVALID;
    if (!ctx->cons_prepared || !ctx->have_catalog)
        return fail(ctx, KP_E_STATE, "kp_consolidate_execute before kp_consolidate_prepare");
    kp_ctx* c = ctx;
    HIPCHK(hipSetDevice(c->device));
    KpCons k = c->cons;
    const int NC = k.n_cand;
    const int nmp = std::max(0, m1 - m0), nsp = std::max(0, s1 - s0);
    const int nprobe = nmp + nsp;
    if (nprobe == 0) return KP_OK;
    const int mode = nmp && nsp ? KP_CONSOLIDATE_BOTH : nmp ? KP_CONSOLIDATE_MULTI : KP_CONSOLIDATE_SINGLE;
    KpDev d = c->dev;
    const int P = d.P, E = d.E, A = d.n_active;
    d.lds_A = 0;  // no quick-accept witness in probes
    d.lds_nstage = A;
    d.profile = 0;
    hipStream_t s = c->stream;
    const std::vector<int32_t>& coff = c->cons_off;
    int maxp = 0;  // ring capacity: pods of the largest probe
    for (int i = s0; i < s1; i++) maxp = std::max(maxp, coff[i + 1] - coff[i]);
    if (m1 > m0) maxp = std::max(maxp, coff[std::min(NC, m1 + 1)]);
    k.mode = mode;
    k.n_probes = nprobe;
    k.probe0 = mode == KP_CONSOLIDATE_SINGLE ? s0 : m0;
    k.n_multi = m1 - m0;
    k.sprobe0 = s0;
    k.ring_cap = std::max(1, c->cons_n_pending + maxp);
    HIPCHK(c->d_cmax0.ensure((size_t)std::max(d.EW, 1) * KP_LDS_AXES));
    k.cmax0 = getenv("KPSIM_CONS_NOSUMMARY") ? nullptr : c->d_cmax0.p;  // diagnostics: no chunk summary
    if (!kp_cons_plan_lds(d, k, KP_LDS_BYTES)) return fail(ctx, KP_E_UNSUPPORTED, "consolidation LDS plan exceeds 160 KB");
    const int occ = std::max(1, std::min(8, KP_LDS_BYTES / std::max(k.lds_bytes, 1)));
    const int workers = std::min(nprobe, 256 * occ);
    if (k.G > 0) {  // per-worker probe topology counts (ProbeTopo); the base counts are read-only in probes
        HIPCHK(c->d_pt_cnt.ensure((size_t)workers * k.G * 64));
        HIPCHK(c->d_pt_known.ensure((size_t)workers * k.G));
        HIPCHK(c->d_pt_hd.ensure((size_t)workers * std::max(k.HG, 1) * (E + 1)));
        k.pt_cnt = c->d_pt_cnt.p;
        k.pt_known = c->d_pt_known.p;
        k.pt_hd = c->d_pt_hd.p;
        k.pt_dgk = c->d_pt_dgk.p;
        k.dec_soff = c->d_dec_soff.p;
        k.dec_moff = c->d_dec_moff.p;
        k.dec_g = c->d_dec_g.p;
        k.dec_v = c->d_dec_v.p;
        k.tg_ha = c->d_tg_ha.p;
        k.hpos0 = c->d_hpos0.p;
        d.tg_cnt = c->d_tg_cnt0.p;
        d.tg_hcnt = c->d_tg_hcnt0.p;
    }
    const auto t0 = clk::now();
    HIPCHK(c->d_ring.ensure((size_t)workers * k.ring_cap));
    HIPCHK(c->d_ring_last.ensure((size_t)workers * k.ring_cap));
    k.relax = d.relax_next ? 1 : 0;  // preference relaxation: relaxed queue entries carry their class and shape
    if (k.relax) {
        HIPCHK(c->d_ring_cls.ensure((size_t)workers * k.ring_cap));
        HIPCHK(c->d_ring_shape.ensure((size_t)workers * k.ring_cap));
        k.ring_cls = c->d_ring_cls.p;
        k.ring_shape = c->d_ring_shape.p;
    }
    HIPCHK(c->d_pnode.ensure((size_t)workers * k.ring_cap));
    HIPCHK(c->d_delta.ensure((size_t)workers * std::max(A, 1) * std::max(E, 1)));
    const size_t pb = (size_t)workers * k.PW;
    if (c->d_pbits.n < pb) {  // kept all-zero between probes by the kernel
        HIPCHK(c->d_pbits.ensure(pb));
        HIPCHK(hipMemsetAsync(c->d_pbits.p, 0, pb * 8, s));
    }
    HIPCHK(c->d_probe_out.ensure(nprobe));
    HIPCHK(hipMemsetAsync(c->d_cons_stats.p, 0, CS_COUNT * sizeof(int64_t), s));
    HIPCHK(hipMemsetAsync(c->d_next.p, 0, 3 * sizeof(int32_t), s));
    HIPCHK(c->d_retry.ensure(nprobe));
    HIPCHK(hipEventRecord(c->ev[0], s));
    if (!c->cons_prep_valid) {
        HIPCHK(hipMemsetAsync(c->d_pend_bits.p, 0, (size_t)k.PW * 8, s));
        if (!c->h_remaining.empty())
            HIPCHK(hipMemcpyAsync(c->d_remaining.p, c->h_remaining.data(), c->h_remaining.size() * sizeof(int64_t),
                                  hipMemcpyHostToDevice, s));
        int32_t* q0 = nullptr;
        if (P > 0) {
            size_t tb = c->sort_temp_bytes;
            HIPCHK(kp_queue_sort(c->d_sort_fields.p, P, c->d_perm_a.p, c->d_perm_b.p, c->d_keys_a.p, c->d_keys_b.p,
                                 c->d_sort_temp.p, &tb, s, &q0));
        }
        d.queue0 = q0;
        HIPCHK(kp_launch_cons_prep(q0, P, c->d_rank.p, c->d_pending.p, c->cons_n_pending, c->d_pend_bits.p, s));
        HIPCHK(kp_launch_class_mask(d, s));
        HIPCHK(kp_launch_template_init(d, s));
        HIPCHK(kp_launch_existing(d, s));
        HIPCHK(kp_launch_cons_chunk_max(d, c->d_cmax0.p, s));
        c->cons_q0 = q0;
        c->cons_prep_valid = true;
    }
    d.queue0 = c->cons_q0;
    HIPCHK(hipEventRecord(c->ev[1], s));
    k.cand_i = c->d_cand_i.p;
    k.cand_off = c->d_cand_off.p;
    k.cand_pods = c->d_cand_pods.p;
    k.cand_price = c->d_cand_price.p;
    k.cand_cap = c->d_cand_cap.p;
    k.rank = c->d_rank.p;
    k.pend_bits = c->d_pend_bits.p;
    k.init_bits = c->d_init.p;
    k.n_pending = c->cons_n_pending;
    k.alloc_act = c->d_alloc_act.p;
    k.ring = c->d_ring.p;
    k.ring_last = c->d_ring_last.p;
    k.pnode = c->d_pnode.p;
    k.delta = c->d_delta.p;
    k.mut_s = c->d_mut_s.p;
    k.mut_m = c->d_mut_m.p;
    if (k.mut) {
        // the MUT variant's node requirement copies: a probe copies a node's digest when a merge first changes it, at
        // most once per node and per pod it places (FULL workers only; the fast variants hand MUT probes over)
        const int fw = std::min(workers, KP_CONS_FULL_WORKERS);
        k.ov_cap = std::max(1, std::min(std::max(E, 1), k.ring_cap));
        HIPCHK(c->d_ov_slot.ensure((size_t)fw * std::max(E, 1)));
        HIPCHK(c->d_ov_hdr.ensure((size_t)fw * k.ov_cap * std::max(d.K, 1)));
        HIPCHK(c->d_ov_words.ensure((size_t)fw * k.ov_cap * std::max(d.DW, 1)));
        k.ov_slot = c->d_ov_slot.p;
        k.ov_hdr = c->d_ov_hdr.p;
        k.ov_words = c->d_ov_words.p;
    }
    k.pbits = c->d_pbits.p;
    k.next_probe = c->d_next.p;
    k.retry = c->d_retry.p;
    k.out = c->d_probe_out.p;
    k.stats = c->d_cons_stats.p;
    k.profile = getenv("KPSIM_PROFILE") ? 1 : 0;
    k.no_fast = getenv("KPSIM_CONS_NOFAST") ? atoi(getenv("KPSIM_CONS_NOFAST")) : 0;  // 1: FULL only, 2: fast only
    if (A > KP_LDS_AXES) k.no_fast = 1;  // more requested axes than the probe registers hold: the FULL variant's serial path
    k.ulist = nullptr;
    k.ulen = nullptr;
    if (nmp > 0 && !getenv("KPSIM_CONS_NOUNION")) {  // diagnostics: KPSIM_CONS_NOUNION=1 builds every probe from bitmaps
        const int nu = std::min(NC, m1 + 1);  // candidates of the call's longest prefix
        HIPCHK(c->d_ubits.ensure(std::max(k.PW, 1)));
        HIPCHK(c->d_rcand.ensure(std::max(P, 1)));
        HIPCHK(c->d_ulen.ensure(1));
        HIPCHK(c->d_ulist.ensure((size_t)std::max(1, coff[nu] - coff[0] + c->cons_n_pending)));
        HIPCHK(kp_launch_multi_union(k, nu, c->d_ubits.p, c->d_rcand.p, c->d_ulist.p, c->d_ulen.p, c->cons_q0, s));
        k.ulist = c->d_ulist.p;
        k.ulen = c->d_ulen.p;
    }
    k.prof_probe = nullptr;
    if (k.profile) {
        HIPCHK(c->d_prof_probe.ensure((size_t)nprobe * KP_CONS_PP));
        HIPCHK(hipMemsetAsync(c->d_prof_probe.p, 0, (size_t)nprobe * KP_CONS_PP * sizeof(int64_t), s));
        k.prof_probe = c->d_prof_probe.p;
    }
    k.rec_i = nullptr;
    k.rec_hdr = nullptr;
    k.rec_words = nullptr;
    if (record) {
        HIPCHK(c->d_rec_i.ensure(4 + 64 + 1));
        HIPCHK(c->d_rec_hdr.ensure(std::max(d.K, 1)));
        HIPCHK(c->d_rec_words.ensure(std::max(d.DW, 1)));
        HIPCHK(hipMemsetAsync(c->d_rec_i.p, 0xff, (4 + 64 + 1) * sizeof(int32_t), s));
        k.rec_i = c->d_rec_i.p;
        k.rec_hdr = c->d_rec_hdr.p;
        k.rec_words = c->d_rec_words.p;
        k.no_fast = 1;
    }
    HIPCHK(c->d_cons_dev.ensure(1));
    HIPCHK(c->d_cons_k.ensure(1));
    HIPCHK(hipMemcpyAsync(c->d_cons_dev.p, &d, sizeof(KpDev), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_cons_k.p, &k, sizeof(KpCons), hipMemcpyHostToDevice, s));
    HIPCHK(kp_launch_consolidate(d, k, workers, s, c->d_cons_dev.p, c->d_cons_k.p));
    HIPCHK(hipEventRecord(c->ev[2], s));
    if (nmp)
        HIPCHK(hipMemcpyAsync(out_multi, c->d_probe_out.p, (size_t)nmp * sizeof(kp_probe_result), hipMemcpyDeviceToHost, s));
    if (nsp)
        HIPCHK(hipMemcpyAsync(out_single, c->d_probe_out.p + nmp, (size_t)nsp * sizeof(kp_probe_result),
                              hipMemcpyDeviceToHost, s));
    int64_t cst[CS_COUNT];
    HIPCHK(hipMemcpyAsync(cst, c->d_cons_stats.p, sizeof cst, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    c->cons_ms[0] = ms;
    HIPCHK(hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
    c->cons_ms[1] = ms;
    c->cons_ms[2] = ns_since(t0) * 1e-6;
    for (int i = 0; i < CS_COUNT; i++) c->cons_stats[i] = cst[i];
    if (k.prof_probe) {  // diagnostics: the probes that bound the pass
        std::vector<int64_t> pp((size_t)nprobe * KP_CONS_PP);
        HIPCHK(hipMemcpy(pp.data(), k.prof_probe, pp.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
        for (int part = 0; part < 2; part++) {
            const int b = part == 0 ? 0 : nmp, e = part == 0 ? nmp : nprobe;
            int arg = -1;
            for (int i = b; i < e; i++)
                if (arg < 0 || pp[(size_t)i * KP_CONS_PP + 2] > pp[(size_t)arg * KP_CONS_PP + 2]) arg = i;
            if (arg >= 0) {
                const int64_t* q = &pp[(size_t)arg * KP_CONS_PP];
                fprintf(stderr, "[kpsim] %s probes %d: longest #%d: %lld cycles (build %lld, placement %lld: window loads %lld, "
                        "chunk prep %lld, node intake %lld over %lld node visits), %lld pods\n",
                        part == 0 ? "multi-node" : "single-node", e - b, arg - b, (long long)q[2], (long long)q[0],
                        (long long)q[1], (long long)q[4], (long long)q[5], (long long)q[6], (long long)q[7], (long long)q[3]);
                fprintf(stderr, "[kpsim]   intake: %lld prefix-sum rounds, %lld scalar steps; %lld pods past the store in %lld "
                        "cycles; NodeClaim %lld cycles, decide %lld cycles; chunk loads %lld, summary skips %lld\n", (long long)q[8],
                        (long long)q[9], (long long)q[11], (long long)q[10], (long long)q[12], (long long)q[13],
                        (long long)q[14], (long long)q[15]);
            }
        }
    }
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

// Probes [b0, b1) of `mode` as a multi-node part [m0, m1) and a single-node part [s0, s1) (BOTH: the multi-node probes
// come first in the caller's numbering).  Multi-device: each part is split into one contiguous shard per device (so the
// long multi-node prefixes spread over the devices instead of all landing on the first), each device runs its two
// shards in one launch from its own host thread, writing into its slices of `results`; counters are summed, device
// times are the max over devices.  Probes are independent, so the gathered vector equals a single-device evaluation.
static kp_status cons_execute(kp_ctx* ctx, int32_t mode, int32_t probe_begin, int32_t probe_end,
                              kp_probe_result* results, int32_t cap_results) try {
    if (!ctx) return KP_E_INVALID;
    if (!ctx->cons_prepared || !ctx->have_catalog)
        return fail(ctx, KP_E_STATE, "kp_consolidate_execute before kp_consolidate_prepare");
    for (kp_ctx* p : ctx->peers)
        if (!p->cons_prepared || !p->have_catalog)
            return fail(ctx, KP_E_STATE, "kp_consolidate_execute: a peer device has no prepared pass");
    if (mode != KP_CONSOLIDATE_SINGLE && mode != KP_CONSOLIDATE_MULTI && mode != KP_CONSOLIDATE_BOTH)
        return fail(ctx, KP_E_INVALID, "unknown consolidation mode");
    const int np = cons_probes(ctx, mode);
    const int b0 = probe_begin > 0 ? probe_begin : 0;
    const int b1 = probe_end > 0 && probe_end < np ? probe_end : np;
    if (b0 > b1) return fail(ctx, KP_E_INVALID, "probe range outside the probe list");
    const int nprobe = b1 - b0;
    if (nprobe > cap_results || (nprobe > 0 && !results)) return fail(ctx, KP_E_BUFFER, "probe results buffer too small");
    if (nprobe == 0) return KP_OK;
    const int nm_all = cons_probes(ctx, KP_CONSOLIDATE_MULTI);
    int m0 = 0, m1 = 0, s0 = 0, s1 = 0;
    if (mode == KP_CONSOLIDATE_MULTI) {
        m0 = b0, m1 = b1;
    } else if (mode == KP_CONSOLIDATE_SINGLE) {
        s0 = b0, s1 = b1;
    } else {
        m0 = std::min(b0, nm_all), m1 = std::min(b1, nm_all);
        s0 = std::max(b0, nm_all) - nm_all, s1 = std::max(b1, nm_all) - nm_all;
    }
    kp_probe_result* rm = results;
    kp_probe_result* rs = results + (m1 - m0);
    if (ctx->peers.empty()) return cons_run(ctx, m0, m1, s0, s1, rm, rs);
    const auto t0 = clk::now();
    const int G = 1 + (int)ctx->peers.size();
    std::vector<kp_ctx*> dev(1, ctx);
    dev.insert(dev.end(), ctx->peers.begin(), ctx->peers.end());
    std::vector<int> ml(G), mh(G), sl(G), sh(G);
    for (int g = 0; g < G; g++) {
        ml[g] = m0 + (int)((int64_t)(m1 - m0) * g / G);
        mh[g] = m0 + (int)((int64_t)(m1 - m0) * (g + 1) / G);
        sl[g] = s0 + (int)((int64_t)(s1 - s0) * g / G);
        sh[g] = s0 + (int)((int64_t)(s1 - s0) * (g + 1) / G);
    }
    std::vector<kp_status> st(G, KP_OK);
    auto run = [&](int g) {
        try {
            st[g] = cons_run(dev[g], ml[g], mh[g], sl[g], sh[g], rm + (ml[g] - m0), rs + (sl[g] - s0));
        } catch (...) {
            st[g] = fail(dev[g], KP_E_INVALID, "consolidation shard: host error");
        }
    };
    std::vector<std::thread> th;
    th.reserve(G - 1);
    for (int g = 1; g < G; g++) th.emplace_back(run, g);
    run(0);
    for (auto& t : th) t.join();
    for (int g = 0; g < G; g++)
        if (st[g] != KP_OK)
            return g == 0 ? st[0] : fail(ctx, st[g], "device " + std::to_string(dev[g]->device) + ": " + dev[g]->err);
    int64_t sum[CS_COUNT] = {};
    double ms0 = 0, ms1 = 0;
    for (int g = 0; g < G; g++) {
        if (mh[g] <= ml[g] && sh[g] <= sl[g]) continue;
        for (int i = 0; i < CS_COUNT; i++) sum[i] += dev[g]->cons_stats[i];
        ms0 = std::max(ms0, dev[g]->cons_ms[0]);
        ms1 = std::max(ms1, dev[g]->cons_ms[1]);
    }
    for (int i = 0; i < CS_COUNT; i++) ctx->cons_stats[i] = sum[i];
    ctx->cons_ms[0] = ms0;
    ctx->cons_ms[1] = ms1;
    ctx->cons_ms[2] = ns_since(t0) * 1e-6;
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_consolidate_execute(kp_ctx* ctx, int32_t mode, int32_t probe_begin, int32_t probe_end,
                                            kp_probe_result* results, int32_t cap_results) try {
    if (!ctx) return KP_E_INVALID;
    const uint64_t gen = ctx->cons_gen;
    const kp_status st = cons_execute(ctx, mode, probe_begin, probe_end, results, cap_results);
    if (st != KP_OK) return st;
    ctx->n_pass_launches++;
    const int np = cons_probes(ctx, mode);
    const int b0 = probe_begin > 0 ? probe_begin : 0;
    const int b1 = probe_end > 0 && probe_end < np ? probe_end : np;
    if (b0 == 0 && b1 == np && gen == ctx->cons_gen) {  // a full pass: kp_consolidate_command can replay it
        ctx->pass_rows.assign(results, results + np);
        ctx->pass_mode = mode;
        ctx->pass_gen = gen;
    }
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_consolidate(kp_ctx* ctx, const kp_consolidate_input* in, kp_probe_result* results,
                                    int32_t cap_results) {
    if (!ctx || !in) return KP_E_INVALID;
    const int np = kp_consolidate_probe_count(in);
    const int b0 = in->probe_begin > 0 ? in->probe_begin : 0;
    const int b1 = in->probe_end > 0 && in->probe_end < np ? in->probe_end : np;
    if (b0 > b1) return fail(ctx, KP_E_INVALID, "probe range outside the probe list");
    if (b1 - b0 > cap_results || (b1 > b0 && !results)) return fail(ctx, KP_E_BUFFER, "probe results buffer too small");
    kp_status st = kp_consolidate_prepare(ctx, in);
    if (st != KP_OK) return st;
    if (b1 == b0) return KP_OK;
    return kp_consolidate_execute(ctx, in->mode, b0, b1, results, cap_results);
}

// firstNConsolidationOption's binary search over the multi-node probe rows (row i = the prefix of i + 2 candidates):
// the largest prefix whose command is DELETE or a REPLACE with options left (row.valid).  Returns the row or -1.
static int replay_multi(const kp_probe_result* r, int n_cand, int max_cand) {
    if (n_cand < 2) return -1;
    int lo = 1, hi = max_cand;
    if (n_cand <= hi) hi = n_cand - 1;
    int best = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        if (r[mid - 1].valid) {
            best = mid - 1;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    return best;
}

static void command_clear(kp_consolidation_command* out) {
    out->decision = KP_DECISION_NONE;
    out->mode = -1;
    out->probe = -1;
    out->first_candidate = 0;
    out->n_candidates = 0;
    out->nodepool = -1;
    out->n_type_ids = 0;
    out->n_reserved = 0;
    out->requirements_needed = 0;
    out->result = kp_probe_result{};
    if (out->requirements && out->cap_requirements > 0) out->requirements[0] = 0;
}

// The replacement NodeClaim of probe `probe` of mode `chosen` (SINGLE / MULTI): the probe re-run on the primary device
// with the read-back on (FULL variant; the pass's timings and counters stay those of the pass), kept per prepared pass
// so that a repeated call (a KP_E_BUFFER retry) copies it.  Fills out's replacement fields and result row.
static kp_status cons_readback(kp_ctx* ctx, int chosen, int probe, kp_consolidation_command* out) {
    if (!(ctx->rec_gen == ctx->cons_gen && ctx->rec_mode == chosen && ctx->rec_probe == probe)) {
        double ms_keep[3];
        int64_t st_keep[CS_COUNT];
        memcpy(ms_keep, ctx->cons_ms, sizeof ms_keep);
        memcpy(st_keep, ctx->cons_stats, sizeof st_keep);
        const uint64_t gen = ctx->cons_gen;
        kp_probe_result again{};
        const bool multi = chosen == KP_CONSOLIDATE_MULTI;
        const kp_status st = multi ? cons_run(ctx, probe, probe + 1, 0, 0, &again, nullptr, true)
                                   : cons_run(ctx, 0, 0, probe, probe + 1, nullptr, &again, true);
        memcpy(ctx->cons_ms, ms_keep, sizeof ms_keep);
        memcpy(ctx->cons_stats, st_keep, sizeof st_keep);
        if (st != KP_OK) return st;
        ctx->n_readbacks++;
        const int K = ctx->K, DW = ctx->DW;
        ctx->rec_h.assign(std::max(K, 1), ReqHdr{});
        ctx->rec_w.assign(std::max(DW, 1), 0);
        HIPCHK(hipMemcpy(ctx->rec_ri, ctx->d_rec_i.p, sizeof ctx->rec_ri, hipMemcpyDeviceToHost));
        if (again.decision == KP_DECISION_REPLACE) {
            HIPCHK(hipMemcpy(ctx->rec_h.data(), ctx->d_rec_hdr.p, (size_t)K * sizeof(ReqHdr), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(ctx->rec_w.data(), ctx->d_rec_words.p, (size_t)DW * sizeof(uint64_t), hipMemcpyDeviceToHost));
        }
        ctx->rec_row = again;
        ctx->rec_gen = gen;
        ctx->rec_mode = chosen;
        ctx->rec_probe = probe;
    }
    const kp_probe_result& row = ctx->rec_row;
    const int32_t* ri = ctx->rec_ri;
    out->mode = chosen;
    out->probe = probe;
    out->first_candidate = chosen == KP_CONSOLIDATE_SINGLE ? probe : 0;
    out->n_candidates = chosen == KP_CONSOLIDATE_SINGLE ? 1 : probe + 2;
    out->result = row;
    out->decision = row.decision;
    if (row.decision != KP_DECISION_REPLACE) return KP_OK;
    if (ri[0] != KP_DECISION_REPLACE || ri[3] != row.n_replacement_types || ri[1] < 0 || ri[1] >= (int)ctx->tmpl_np.size())
        return fail(ctx, KP_E_DEVICE, "consolidation read-back: inconsistent replacement record");
    std::vector<ReqHdr> h = ctx->rec_h;
    std::vector<uint64_t> w = ctx->rec_w;
    out->nodepool = ctx->tmpl_np[ri[1]];
    out->n_reserved = ri[4 + 64];
    // the replacement was priced as spot: Requirements.Add(capacity-type In [spot]) (consolidation.go)
    if (ri[2] && ctx->key_ct >= 0) {
        const int kct = ctx->key_ct;
        int wo = 0;
        for (int k = 0; k < kct; k++) wo += std::max(1, ((int)ctx->sol.keys[k].vals.size() + 63) / 64);
        const int nwk = std::max(1, ((int)ctx->sol.keys[kct].vals.size() + 63) / 64);
        const int vs = ctx->sol.keys[kct].find("spot");
        ReqHdr& hc = h[kct];
        const uint32_t keep_min = hc.flags & RF_MIN;
        hc.flags = RF_DEF | keep_min;
        hc.gt = hc.lt = 0;
        for (int i = 0; i < nwk; i++) w[wo + i] = 0;
        if (vs >= 0) w[wo + vs / 64] |= 1ull << (vs % 64);
    }
    const int n = ri[3];
    out->n_type_ids = n;
    const std::string txt = reqs_text(ctx, h.data(), w.data());
    out->requirements_needed = (int64_t)txt.size() + 1;
    bool small = false;
    for (int i = 0; i < n; i++) {
        if (i < out->cap_type_ids && out->type_ids) out->type_ids[i] = ri[4 + i];
        else small = true;
    }
    if (out->requirements && out->cap_requirements >= (int64_t)txt.size() + 1)
        memcpy(out->requirements, txt.c_str(), txt.size() + 1);
    else
        small = true;
    return small ? fail(ctx, KP_E_BUFFER, "consolidation command: replacement buffers too small") : KP_OK;
}

extern "C" kp_status kp_consolidate_command(kp_ctx* ctx, int32_t mode, kp_consolidation_command* out) try {
    if (!ctx || !out) return KP_E_INVALID;
    if (mode != KP_CONSOLIDATE_SINGLE && mode != KP_CONSOLIDATE_MULTI && mode != KP_CONSOLIDATE_BOTH)
        return fail(ctx, KP_E_INVALID, "unknown consolidation mode");
    if (!ctx->cons_prepared || !ctx->have_catalog)
        return fail(ctx, KP_E_STATE, "kp_consolidate_command before kp_consolidate_prepare");
    command_clear(out);
    const int NC = ctx->cons.n_cand, mx = ctx->cons_max_candidates;
    const int nm = cons_probes(ctx, KP_CONSOLIDATE_MULTI), np = cons_probes(ctx, mode);
    // the probe rows: the last full pass of this prepared pass when it covers `mode` (a BOTH pass covers either),
    // else one pass now
    const bool have = ctx->pass_gen == ctx->cons_gen && (ctx->pass_mode == mode || ctx->pass_mode == KP_CONSOLIDATE_BOTH);
    if (!have && np > 0) {
        std::vector<kp_probe_result> res(np);
        const kp_status st = kp_consolidate_execute(ctx, mode, 0, np, res.data(), np);
        if (st != KP_OK) return st;
    }
    const bool both_rows = ctx->pass_mode == KP_CONSOLIDATE_BOTH;
    const kp_probe_result* mrows = ctx->pass_rows.data();                                  // multi-node rows
    const kp_probe_result* srows = ctx->pass_rows.data() + (both_rows ? nm : 0);           // single-node rows
    // the disruption controller's method order: multi-node (binary search), then single-node (first non-no-op)
    int chosen = -1, probe = -1;
    if (mode != KP_CONSOLIDATE_SINGLE && np > 0) {
        probe = replay_multi(mrows, NC, mx);
        if (probe >= 0) chosen = KP_CONSOLIDATE_MULTI;
    }
    if (chosen < 0 && mode != KP_CONSOLIDATE_MULTI && np > 0) {
        for (int i = 0; i < NC; i++)
            if (srows[i].decision != KP_DECISION_NONE) {
                probe = i;
                chosen = KP_CONSOLIDATE_SINGLE;
                break;
            }
    }
    if (chosen < 0) return KP_OK;
    const kp_probe_result row = chosen == KP_CONSOLIDATE_MULTI ? mrows[probe] : srows[probe];
    out->mode = chosen;
    out->probe = probe;
    out->first_candidate = chosen == KP_CONSOLIDATE_SINGLE ? probe : 0;
    out->n_candidates = chosen == KP_CONSOLIDATE_SINGLE ? 1 : probe + 2;
    out->result = row;
    out->decision = row.decision;
    if (row.decision != KP_DECISION_REPLACE) return KP_OK;
    const kp_status st = cons_readback(ctx, chosen, probe, out);
    if (st != KP_OK && st != KP_E_BUFFER) return st;
    if (out->result.decision != row.decision || out->result.n_replacement_types != row.n_replacement_types)
        return fail(ctx, KP_E_DEVICE, "kp_consolidate_command: the read-back run disagrees with the pass");
    return st;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_consolidate_replacement(kp_ctx* ctx, int32_t mode, int32_t probe, kp_consolidation_command* out) try {
    if (!ctx || !out) return KP_E_INVALID;
    if (mode != KP_CONSOLIDATE_SINGLE && mode != KP_CONSOLIDATE_MULTI)
        return fail(ctx, KP_E_INVALID, "kp_consolidate_replacement: mode must be SINGLE or MULTI");
    if (!ctx->cons_prepared || !ctx->have_catalog)
        return fail(ctx, KP_E_STATE, "kp_consolidate_replacement before kp_consolidate_prepare");
    if (probe < 0 || probe >= cons_probes(ctx, mode)) return fail(ctx, KP_E_INVALID, "probe out of range");
    command_clear(out);
    return cons_readback(ctx, mode, probe, out);
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_consolidate_stats(kp_ctx* ctx, double* ms, int64_t* counters, int32_t n_counters) {
    if (!ctx) return KP_E_INVALID;
    if (ms)
        for (int i = 0; i < 3; i++) ms[i] = ctx->cons_ms[i];
    if (counters)
        for (int i = 0; i < n_counters && i < CS_COUNT + 2; i++)
            counters[i] = i < CS_COUNT ? ctx->cons_stats[i] : i == CS_COUNT ? ctx->n_pass_launches : ctx->n_readbacks;
    return KP_OK;
}

// ---------------------------------------------------------------------------------------------
// launch selection (kp_launch_select): filter.go chain + Truncate + getCapacityType + getOverrides' offering side
// ---------------------------------------------------------------------------------------------
static kp_status upload_launch_tables(kp_ctx* c, const kp_catalog_view* v, const std::vector<uint8_t>& avail) {
    kp_ctx* ctx = c;  // HIPCHK reports through ctx
    const int T = c->T, O = v->n_offerings, KO = v->n_offering_keys;
    c->launch_ok = true;
    c->launch_err.clear();
    c->l_off_begin.assign(T + 1, 0);
    for (int o = 0; o < O; o++) {
        if (o > 0 && v->offering_type[o] < v->offering_type[o - 1])
            return fail(c, KP_E_INVALID, "offering rows must be grouped by type (offering_type non-decreasing)");
        c->l_off_begin[v->offering_type[o] + 1]++;
    }
    for (int t = 0; t < T; t++) {
        if (c->l_off_begin[t + 1] > KL_MAX_OFF) {
            c->launch_ok = false;
            c->launch_err = "more than 64 offerings on one instance type";
        }
        c->l_off_begin[t + 1] += c->l_off_begin[t];
    }
    const int roles[KL_ROLES] = {c->key_zone, c->key_ct, c->key_zoneid, c->key_resvid, c->key_resvtype};
    c->l_off_val.assign((size_t)KL_ROLES * O, KL_V_ABSENT);
    c->l_ct.assign(O, KP_CT_ON_DEMAND);
    c->l_rt.assign(O, -1);
    c->l_rcap.assign(O, 0);
    c->l_price.assign(O, 0.0);
    c->l_avail = avail;
    for (int o = 0; o < O; o++) {
        c->l_price[o] = v->offering_price[o];
        c->l_rcap[o] = v->offering_reservation_capacity ? v->offering_reservation_capacity[o] : 0;
        for (int k = 0; k < KO; k++) {
            const int key = c->cat.find_key(normalize(v->offering_keys[k]));
            int r = -1;
            for (int j = 0; j < KL_ROLES; j++)
                if (roles[j] == key && key >= 0) r = j;
            if (r < 0) continue;
            const int st = v->offering_label_state[(size_t)o * KO + k];
            int val = KL_V_ABSENT;
            if (st == KP_LABEL_DOES_NOT_EXIST) val = KL_V_DNE;
            else if (st == KP_LABEL_IN) val = c->cat.keys[key].id(v->offering_label_values[(size_t)o * KO + k]);
            c->l_off_val[(size_t)r * O + o] = val;
            if (st != KP_LABEL_IN) continue;
            const char* s = v->offering_label_values[(size_t)o * KO + k];
            if (r == KL_ROLE_CT) {
                if (!strcmp(s, "on-demand")) c->l_ct[o] = KP_CT_ON_DEMAND;
                else if (!strcmp(s, "spot")) c->l_ct[o] = KP_CT_SPOT;
                else if (!strcmp(s, "reserved")) c->l_ct[o] = KP_CT_RESERVED;
                else return fail(c, KP_E_INVALID, "unknown capacity type on an offering");
            } else if (r == KL_ROLE_RESVTYPE) {
                // v1.CapacityReservationType("").Values(); filter.go:148 panics on anything else
                if (!strcmp(s, "default")) c->l_rt[o] = 0;
                else if (!strcmp(s, "capacity-block")) c->l_rt[o] = 1;
                else return fail(c, KP_E_INVALID, "unknown capacity-reservation-type on an offering");
            }
        }
    }
    // ExoticInstanceTypeFilter's per-type test (filter.go:294-312): a "metal" size, or accelerator capacity
    c->l_exotic.assign(T, 0);
    const int ksize = c->cat.find_key("karpenter.k8s.aws/instance-size");
    const char* accel[] = {"aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "amd.com/gpu", "nvidia.com/gpu",
                           "habana.ai/gaudi"};
    const int KL = v->n_label_keys;
    for (int t = 0; t < T; t++) {
        bool ex = false;
        for (int k = 0; k < KL && !ex; k++) {
            if (ksize < 0 || c->cat.find_key(normalize(v->label_keys[k])) != ksize) continue;
            if (v->label_state[(size_t)t * KL + k] != KP_LABEL_IN) continue;
            for (int i = v->label_offsets[(size_t)t * KL + k]; i < v->label_offsets[(size_t)t * KL + k + 1]; i++)
                if (strstr(v->label_values[i], "metal")) ex = true;
        }
        for (int r = 0; r < c->R && !ex; r++)
            for (auto* a : accel)
                if (c->resource_names[r] == a && v->capacity[(size_t)t * c->R + r] != 0) ex = true;
        c->l_exotic[t] = ex;
    }
    hipStream_t s = c->stream;
    HIPCHK(c->d_l_off_begin.upload(c->l_off_begin, s));
    HIPCHK(c->d_l_off_val.upload(c->l_off_val, s));
    HIPCHK(c->d_l_ct.upload(c->l_ct, s));
    HIPCHK(c->d_l_rt.upload(c->l_rt, s));
    HIPCHK(c->d_l_rcap.upload(c->l_rcap, s));
    HIPCHK(c->d_l_price.upload(c->l_price, s));
    HIPCHK(c->d_l_avail.upload(c->l_avail, s));
    HIPCHK(c->d_l_exotic.upload(c->l_exotic, s));
    return KP_OK;
}

namespace {
// scheduling.Requirement in string space (requirement.go: NewRequirementWithFlexibility, Intersection, Has, Operator)
struct SReq {
    bool complement = false;
    std::set<std::string> vals;
    bool has_gt = false, has_lt = false;
    int64_t gt = 0, lt = 0;
    bool has_min = false;
    int minv = 0;
    bool within(const std::string& v) const {
        if (!has_gt && !has_lt) return true;
        int64_t x = 0;
        if (!go_atoi(v.c_str(), x)) return false;
        if (has_gt && gt >= x) return false;
        if (has_lt && lt <= x) return false;
        return true;
    }
    bool has(const std::string& v) const { return (complement ? !vals.count(v) : vals.count(v) > 0) && within(v); }
    int op() const {  // 0 In, 1 NotIn, 2 Exists, 3 DoesNotExist
        if (complement) return vals.empty() ? 2 : 1;
        return vals.empty() ? 3 : 0;
    }
};
SReq sreq_new(const kp_requirement& r) {
    SReq q;
    q.complement = !(r.op == KP_OP_IN || r.op == KP_OP_DOES_NOT_EXIST);
    if (r.op == KP_OP_IN || r.op == KP_OP_NOT_IN)
        for (int j = 0; j < r.n_values; j++) q.vals.insert(r.values[j] ? r.values[j] : "");
    if (r.op == KP_OP_GT || r.op == KP_OP_LT) {
        int64_t x = 0;
        go_atoi(r.n_values > 0 && r.values[0] ? r.values[0] : "", x);
        (r.op == KP_OP_GT ? q.has_gt : q.has_lt) = true;
        (r.op == KP_OP_GT ? q.gt : q.lt) = x;
    }
    q.has_min = r.min_values >= 0;
    q.minv = r.min_values;
    return q;
}
SReq sreq_intersection(const SReq& a, const SReq& b) {
    SReq o;
    o.complement = a.complement && b.complement;
    o.has_gt = a.has_gt || b.has_gt;
    o.gt = (a.has_gt && b.has_gt) ? std::max(a.gt, b.gt) : (a.has_gt ? a.gt : b.gt);
    o.has_lt = a.has_lt || b.has_lt;
    o.lt = (a.has_lt && b.has_lt) ? std::min(a.lt, b.lt) : (a.has_lt ? a.lt : b.lt);
    o.has_min = a.has_min || b.has_min;
    o.minv = (a.has_min && b.has_min) ? std::max(a.minv, b.minv) : (a.has_min ? a.minv : b.minv);
    if (o.has_gt && o.has_lt && o.gt >= o.lt) {
        SReq d;
        d.has_min = o.has_min;
        d.minv = o.minv;
        return d;
    }
    std::set<std::string> vs;
    if (a.complement && b.complement) {
        vs = a.vals;
        vs.insert(b.vals.begin(), b.vals.end());
    } else if (a.complement) {
        for (auto& x : b.vals)
            if (!a.vals.count(x)) vs.insert(x);
    } else if (b.complement) {
        for (auto& x : a.vals)
            if (!b.vals.count(x)) vs.insert(x);
    } else {
        for (auto& x : a.vals)
            if (b.vals.count(x)) vs.insert(x);
    }
    for (auto& x : vs)
        if (o.within(x)) o.vals.insert(x);
    if (!o.complement) o.has_gt = o.has_lt = false;
    return o;
}

// The same requirement in the catalog's value-id space (launch-request encoding): `ids` are the values the catalog
// dictionary of key kc knows (sorted), `unk` the others (kept by name only — they decide whether a set is empty).
struct IReq {
    int kc = -1;          // catalog key, -1 when no type or offering carries it
    const char* name = "";  // normalised key (the request's string or a static alias target)
    bool comp = false;
    std::vector<int> ids;
    std::vector<std::string> unk;
    bool has_gt = false, has_lt = false;
    int64_t gt = 0, lt = 0;
    bool has_min = false;
    int minv = 0;
    int op() const {  // 0 In, 1 NotIn, 2 Exists, 3 DoesNotExist
        const bool empty = ids.empty() && unk.empty();
        if (comp) return empty ? 2 : 1;
        return empty ? 3 : 0;
    }
};
const char* const kCtNames[3] = {"on-demand", "spot", "reserved"};
bool ireq_within(const IReq& q, const std::string& v) {
    if (!q.has_gt && !q.has_lt) return true;
    int64_t x = 0;
    if (!go_atoi(v.c_str(), x)) return false;
    if (q.has_gt && q.gt >= x) return false;
    if (q.has_lt && q.lt <= x) return false;
    return true;
}
// fills q in place (its vectors keep their capacity across requests)
void ireq_fill(const kp_ctx* c, const kp_requirement& r, IReq& q) {
    q.name = normalize_c(r.key);
    q.kc = c->cat.find_key_fast(q.name);
    q.comp = !(r.op == KP_OP_IN || r.op == KP_OP_DOES_NOT_EXIST);
    q.ids.clear();
    q.unk.clear();
    q.has_gt = q.has_lt = false;
    q.gt = q.lt = 0;
    if (r.op == KP_OP_IN || r.op == KP_OP_NOT_IN) {
        const KeyDict* kd = q.kc >= 0 ? &c->cat.keys[q.kc] : nullptr;
        q.ids.reserve(r.n_values);
        for (int j = 0; j < r.n_values; j++) {
            const char* v = r.values[j] ? r.values[j] : "";
            const int id = kd ? kd->find_fast(v) : -1;
            if (id >= 0) q.ids.push_back(id);
            else q.unk.emplace_back(v);
        }
        // ids stay in request order (duplicates allowed): the bitset build ORs them; ireq_norm sorts them for the set
        // algebra of a repeated key
        std::sort(q.unk.begin(), q.unk.end());
        q.unk.erase(std::unique(q.unk.begin(), q.unk.end()), q.unk.end());
    }
    if (r.op == KP_OP_GT || r.op == KP_OP_LT) {
        int64_t x = 0;
        go_atoi(r.n_values > 0 && r.values[0] ? r.values[0] : "", x);
        (r.op == KP_OP_GT ? q.has_gt : q.has_lt) = true;
        (r.op == KP_OP_GT ? q.gt : q.lt) = x;
    }
    q.has_min = r.min_values >= 0;
    q.minv = r.min_values;
}
void ireq_norm(IReq& q) {
    std::sort(q.ids.begin(), q.ids.end());
    q.ids.erase(std::unique(q.ids.begin(), q.ids.end()), q.ids.end());
}
template <class V>
V set_op(const V& a, const V& b, int how) {  // 0 union, 1 a \ b, 2 a ∩ b (sorted inputs)
    V o;
    if (how == 0) std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
    else if (how == 1) std::set_difference(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
    else std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
    return o;
}
// Requirement.Intersection (same rules as sreq_intersection, in value-id space)
IReq ireq_intersection(const kp_ctx* c, const IReq& a, const IReq& b) {
    IReq o;
    o.kc = a.kc;
    o.name = a.name;
    o.comp = a.comp && b.comp;
    o.has_gt = a.has_gt || b.has_gt;
    o.gt = (a.has_gt && b.has_gt) ? std::max(a.gt, b.gt) : (a.has_gt ? a.gt : b.gt);
    o.has_lt = a.has_lt || b.has_lt;
    o.lt = (a.has_lt && b.has_lt) ? std::min(a.lt, b.lt) : (a.has_lt ? a.lt : b.lt);
    o.has_min = a.has_min || b.has_min;
    o.minv = (a.has_min && b.has_min) ? std::max(a.minv, b.minv) : (a.has_min ? a.minv : b.minv);
    if (o.has_gt && o.has_lt && o.gt >= o.lt) {
        IReq d;
        d.kc = a.kc;
        d.name = a.name;
        d.has_min = o.has_min;
        d.minv = o.minv;
        return d;
    }
    const int how = (a.comp && b.comp) ? 0 : 2;
    if (a.comp && !b.comp) {
        o.ids = set_op(b.ids, a.ids, 1);
        o.unk = set_op(b.unk, a.unk, 1);
    } else if (b.comp && !a.comp) {
        o.ids = set_op(a.ids, b.ids, 1);
        o.unk = set_op(a.unk, b.unk, 1);
    } else {
        o.ids = set_op(a.ids, b.ids, how);
        o.unk = set_op(a.unk, b.unk, how);
    }
    if (o.has_gt || o.has_lt) {  // values outside the bounds are dropped
        const std::vector<std::string>* vals = o.kc >= 0 ? &c->cat.keys[o.kc].vals : nullptr;
        std::vector<int> ids;
        for (int v : o.ids)
            if (ireq_within(o, (*vals)[v])) ids.push_back(v);
        o.ids.swap(ids);
        std::vector<std::string> unk;
        for (auto& x : o.unk)
            if (ireq_within(o, x)) unk.push_back(x);
        o.unk.swap(unk);
    }
    if (!o.comp) o.has_gt = o.has_lt = false;
    return o;
}
// Requirement.Has for a value given by id (or by name when the dictionary does not know it, id < 0)
bool ireq_has(const kp_ctx* c, const IReq& q, int id, const char* name) {
    bool in;
    if (id >= 0) in = std::find(q.ids.begin(), q.ids.end(), id) != q.ids.end();
    else in = std::binary_search(q.unk.begin(), q.unk.end(), std::string(name));
    return (q.comp ? !in : in) && ireq_within(q, name);
}
}  // namespace

extern "C" kp_status kp_launch_select(kp_ctx* ctx, int32_t n, const kp_launch_request* requests,
                                      int32_t max_instance_types, kp_launch_result* results, int32_t* type_ids,
                                      int32_t cap_type_ids, int32_t* override_offerings, int32_t cap_overrides) try {
    if (!ctx || n < 0 || (n > 0 && (!requests || !results))) return KP_E_INVALID;
    if (!ctx->have_catalog) return fail(ctx, KP_E_STATE, "kp_launch_select before kp_catalog_upload");
    if (!ctx->launch_ok) return fail(ctx, KP_E_UNSUPPORTED, ctx->launch_err);
    const int M = max_instance_types;
    if (M < 1 || M > 64) return fail(ctx, KP_E_UNSUPPORTED, "max_instance_types must be in 1..64 (instance.go:62 uses 60)");
    const auto t0 = clk::now();
    HIPCHK(hipSetDevice(ctx->device));
    kp_ctx* c = ctx;
    const int T = c->T, R = c->R, Kc = c->Kcat;
    // Requests are encoded independently (NewNodeSelectorRequirementsWithMinValues + digest per NodeClaim), so the
    // batch is split over host threads into chunk-local tables that are concatenated with their offsets rebased.
    HIPCHK(c->p_l_req.ensure(std::max(1, n)));
    HIPCHK(c->p_l_rq.ensure((size_t)std::max(1, n) * R));
    KlReq* const reqs = c->p_l_req.p;
    int64_t* const rq = c->p_l_rq.p;
    memset(rq, 0, (size_t)std::max(1, n) * R * sizeof(int64_t));
    const int roles[KL_ROLES] = {c->key_zone, c->key_ct, c->key_zoneid, c->key_resvid, c->key_resvtype};
    struct Chunk {
        std::vector<KlKey> keys;
        std::vector<KlMinKey> mins;
        std::vector<uint64_t> words;
        std::vector<IReq> scratch;
        std::vector<uint8_t> constrained;
        kp_status st = KP_OK;
        std::string msg;
    };
    for (int x = 0; x < 3; x++) c->ct_vid[x] = c->key_ct >= 0 ? c->cat.keys[c->key_ct].find(kCtNames[x]) : -1;
    int nthr = std::max(1, std::min<int>({16, (int)std::thread::hardware_concurrency(), (n + 255) / 256}));
    if (const char* e = getenv("KPSIM_LAUNCH_THREADS")) nthr = std::max(1, std::min(nthr, atoi(e)));  // diagnostics
    // per calling thread, reused across calls: the chunk tables and requirement slots keep their capacity, so the
    // encoding threads do not contend in malloc
    // (a named reference: the worker threads must reach the calling thread's instance, not their own)
    static thread_local std::vector<Chunk> tl_chunks;
    std::vector<Chunk>& chunks = tl_chunks;
    if ((int)chunks.size() < nthr) chunks.resize(nthr);
    for (auto& ch : chunks) {
        ch.st = KP_OK;
        ch.msg.clear();
    }
    // catalog keys that are well-known labels (undefined on a request: no constraint), computed once per call
    std::vector<uint8_t> wk(Kc, 0);
    for (int kc = 0; kc < Kc; kc++) wk[kc] = well_known(c->cat.keys[kc].name) ? 1 : 0;
    auto encode_one = [&](int i, Chunk& ch) -> bool {
        std::vector<KlKey>& keys = ch.keys;
        std::vector<KlMinKey>& mins = ch.mins;
        std::vector<uint64_t>& words = ch.words;
        auto err = [&](kp_status st, const char* m) {
            ch.st = st;
            ch.msg = m;
            return false;
        };
        const kp_launch_request& lr = requests[i];
        if (lr.n_requirements < 0 || (lr.n_requirements > 0 && !lr.requirements)) return err(KP_E_INVALID, "bad request");
        // NewNodeSelectorRequirementsWithMinValues: Add = intersect per key, in catalog value-id space (values no type
        // or offering carries are kept by name only: they decide whether a set is empty)
        // ch.scratch holds reusable IReq slots: the first nm are this request's merged requirements
        std::vector<IReq>& slots = ch.scratch;
        size_t nm = 0;
        for (int j = 0; j < lr.n_requirements; j++) {
            const kp_requirement& r = lr.requirements[j];
            if (!r.key || r.op < 0 || r.op > 5) return err(KP_E_INVALID, "bad requirement");
            if (nm == slots.size()) slots.emplace_back();
            IReq& q = slots[nm];
            ireq_fill(c, r, q);
            IReq* hit = nullptr;
            for (size_t x = 0; x < nm; x++)
                if (slots[x].kc == q.kc && (q.kc >= 0 || !strcmp(slots[x].name, q.name))) hit = &slots[x];
            if (hit) {
                ireq_norm(q);
                ireq_norm(*hit);
                *hit = ireq_intersection(c, q, *hit);
            }
            else nm++;
        }
        std::sort(slots.begin(), slots.begin() + nm, [](const IReq& a, const IReq& b) { return strcmp(a.name, b.name) < 0; });
        struct View {  // the merged requirements of this request
            const IReq* b;
            const IReq* e;
            const IReq* begin() const { return b; }
            const IReq* end() const { return e; }
        } m{slots.data(), slots.data() + nm};
        if (lr.requests)
            for (int r = 0; r < R; r++) rq[(size_t)i * R + r] = lr.requests[r];
        KlReq& q = reqs[i];
        q = KlReq{};
        q.key_off = (int)keys.size();
        int woff_of[KL_ROLES];
        for (int r = 0; r < KL_ROLES; r++) woff_of[r] = -1;
        const IReq* role_req[KL_ROLES] = {};
        std::vector<uint8_t>& constrained = ch.constrained;
        constrained.assign(Kc, 0);
        for (const IReq& sq : m) {
            const int kc = sq.kc;
            if (kc < 0) continue;  // no type or offering carries the key: absent on both sides, never constrains
            constrained[kc] = 1;
            const KeyDict& kd = c->cat.keys[kc];
            const int nv = (int)kd.vals.size();
            const int woff = (int)words.size();
            words.resize(words.size() + std::max<size_t>(1, (nv + 63) / 64), 0ull);
            // bit v ⇔ Has(vals[v]); In sets visit only their own values, complements start full and clear theirs
            if (!sq.comp) {
                for (int v : sq.ids) words[woff + v / 64] |= 1ull << (v % 64);
            } else {
                const bool bounded = sq.has_gt || sq.has_lt;
                for (int vv = 0; vv < nv; vv++)
                    if (!bounded || ireq_within(sq, kd.vals[vv])) words[woff + vv / 64] |= 1ull << (vv % 64);
                for (int v : sq.ids) words[woff + v / 64] &= ~(1ull << (v % 64));
            }
            const int op = sq.op();
            KlKey kk{kc, c->cat_multi[kc], 0u, woff};
            kk.flags = (c->cat_kflags[kc] & KF_CAT_MULTI) ? KLK_MULTI : KLK_SINGLE;
            if (op == 1 || op == 3) kk.flags |= KLK_DNE_OK;
            if (c->cat_kflags[kc] != 0) keys.push_back(kk);
            for (int r = 0; r < KL_ROLES; r++)
                if (roles[r] == kc) {
                    woff_of[r] = woff;
                    role_req[r] = &sq;
                }
        }
        q.n_keys = (int)keys.size() - q.key_off;
        q.und_off = (int)keys.size();
        for (int kc = 0; kc < Kc; kc++) {
            if (c->cat_kflags[kc] == 0 || constrained[kc] || wk[kc]) continue;
            KlKey kk{kc, c->cat_multi[kc], (c->cat_kflags[kc] & KF_CAT_MULTI) ? KLK_MULTI : KLK_SINGLE, 0};
            keys.push_back(kk);
        }
        q.n_und = (int)keys.size() - q.und_off;
        for (int r = 0; r < KL_ROLES; r++) {
            const int kc = roles[r];
            KlRole& ro = q.role[r];
            ro = KlRole{KLR_PASS, 0u, 0, 0};
            if (kc < 0) continue;
            if (woff_of[r] >= 0) {
                ro.mode = KLR_CONSTRAINED;
                ro.woff = woff_of[r];
                const int op = role_req[r]->op();
                if (op == 1 || op == 3) ro.flags = KLK_DNE_OK;
            } else if (!wk[kc]) {
                ro.mode = KLR_FAIL_IN;
            }
        }
        const IReq* ct = nullptr;
        for (const IReq& x : m)
            if (c->key_ct >= 0 ? x.kc == c->key_ct : !strcmp(x.name, "karpenter.sh/capacity-type")) ct = &x;
        for (int x = 0; x < 3; x++) q.ct_has[x] = ct == nullptr ? 1 : (ireq_has(c, *ct, c->ct_vid[x], kCtNames[x]) ? 1 : 0);
        q.min_off = (int)mins.size();
        for (const IReq& sq : m) {
            if (!sq.has_min) continue;
            q.has_min = 1;
            const int kc = sq.kc;
            KlMinKey mk{-1, -1, 0, sq.minv};
            if (kc >= 0 && c->cat_kflags[kc] != 0) {
                mk.k = kc;
                mk.mi = (c->cat_kflags[kc] & KF_CAT_MULTI) ? c->cat_multi[kc] : -1;
                mk.nvals = (int)c->cat.keys[kc].vals.size();
                if (mk.nvals > KP_MAX_MIN_WORDS * 64) return err(KP_E_UNSUPPORTED, "minValues key with > 4096 values");
            } else {
                mk.k = 0;  // no type carries the key: zero distinct values
                mk.mi = -1;
                mk.nvals = 0;
                if (mk.minv > 0) mk.minv = INT32_MAX;
            }
            mins.push_back(mk);
        }
        q.n_min = (int)mins.size() - q.min_off;
        return true;
    };
    // Pipeline over sub-batches: sub-batch b is encoded on the host threads while the kernel of b-1 runs, and the
    // results of b-1 are expanded once its download has landed.  The request rows (KlReq, requests) and the result
    // rows live at their batch positions; the key / minValues / word tables of sub-batch b go to staging set b & 1,
    // which is free again because sub-batch b-2's download (queued behind its kernel) was waited for before b is
    // encoded.  Sub-batch b runs on stream b & 1, so a kernel's start overlaps the previous kernel's tail of long
    // workgroups.
    // two halves measured best on MI355X for the 10k config-5 batch (call 4.3 -> 3.1 ms; each extra launch costs ~0.17 ms
    // of kernel ramp and tail, and the host encoding of a half outlasts the kernel of the other)
    int nsub = n >= 4096 ? 2 : 1;
    if (const char* e = getenv("KPSIM_LAUNCH_SUB")) nsub = std::max(1, std::min({KL_MAX_SUB, atoi(e), std::max(1, n)}));
    const auto sub_begin = [&](int b) { return (int)((int64_t)n * b / nsub); };
    if (nsub > 1 && !c->lstream2) HIPCHK(hipStreamCreateWithFlags(&c->lstream2, hipStreamNonBlocking));
    hipStream_t s = c->stream;
    if (n > 0) {
        HIPCHK(c->d_l_req.ensure((size_t)n));
        HIPCHK(c->d_l_rq.ensure((size_t)n * R));
        HIPCHK(c->d_l_hdr.ensure((size_t)n * KL_HDR));
        HIPCHK(c->d_l_types.ensure((size_t)n * M));
        HIPCHK(c->d_l_over.ensure((size_t)n * M));
    }
    HIPCHK(c->p_l_hdr.ensure((size_t)std::max(1, n) * KL_HDR));
    HIPCHK(c->p_l_types.ensure((size_t)std::max(1, n) * M));
    HIPCHK(c->p_l_over.ensure((size_t)std::max(1, n) * M));
    for (auto& e : c->lev)
        if (!e) HIPCHK(hipEventCreate(&e));
    KpLaunch g0{};
    g0.T = T;
    g0.TW = c->TW;
    g0.R = R;
    g0.M = M;
    g0.type_val = c->d_type_val.p;
    g0.multi_mask = c->d_multi_mask.p;
    g0.dne_mask = c->d_dne_mask.p;
    g0.alloc = c->d_alloc.p;
    g0.name_rank = c->d_name_rank.p;
    g0.exotic = c->d_l_exotic.p;
    g0.off_begin = c->d_l_off_begin.p;
    g0.off_val = c->d_l_off_val.p;
    g0.ct_code = c->d_l_ct.p;
    g0.rt_code = c->d_l_rt.p;
    g0.off_price = c->d_l_price.p;
    g0.off_avail = c->d_l_avail.p;
    g0.off_rcap = c->d_l_rcap.p;
    const int32_t* const hdr = c->p_l_hdr.p;
    const int32_t* const tys = c->p_l_types.p;
    const uint64_t* const ov = c->p_l_over.p;
    // result rows: counts first (type_offset / override_offset are prefix sums), then the lists, per thread range
    std::vector<int64_t> toff(n + 1, 0), ooff(n + 1, 0);
    bool host_err = false;  // a worker task threw (reported as KP_E_INVALID once the streams are idle)
    auto par = [&](int i0, int i1, auto fn) {  // fn(a, b) over contiguous ranges of [i0, i1) (the ctx's worker threads)
        const int k = std::max(1, std::min(nthr, (i1 - i0) / 256));
        if (k == 1) {
            fn(i0, i1);
            return;
        }
        if (!c->pool.run(k, [&](int ti) { fn(i0 + (int)((int64_t)(i1 - i0) * ti / k), i0 + (int)((int64_t)(i1 - i0) * (ti + 1) / k)); }))
            host_err = true;
    };
    double ms_enc = 0, ms_up = 0, ms_wait = 0, ms_exp = 0;
    float kms_sum = 0.f;
    std::pair<float, float> span[KL_MAX_SUB];  // kernel intervals after the first kernel's start (device busy time)
    auto ms_between = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    auto expand = [&](int b) -> hipError_t {
        const auto tw = clk::now();
        hipError_t he = hipEventSynchronize(c->lev[3 * b + 2]);
        float k = 0.f;
        if (he == hipSuccess) he = hipEventElapsedTime(&k, c->lev[3 * b], c->lev[3 * b + 1]);
        float k0 = 0.f;
        if (he == hipSuccess && b > 0) he = hipEventElapsedTime(&k0, c->lev[0], c->lev[3 * b]);
        if (he != hipSuccess) return he;
        kms_sum += k;
        span[b] = {k0, k0 + k};
        const auto tx = clk::now();
        ms_wait += ms_between(tw, tx);
        const int s0 = sub_begin(b), s1 = sub_begin(b + 1);
        par(s0, s1, [&](int i0, int i1) {
            for (int i = i0; i < i1; i++) {
                const int nt = hdr[(size_t)i * KL_HDR + 3];
                int64_t no = 0;
                for (int k = 0; k < nt; k++) no += __builtin_popcountll(ov[(size_t)i * M + k]);
                toff[i + 1] = nt;
                ooff[i + 1] = no;
            }
        });
        for (int i = s0; i < s1; i++) {
            toff[i + 1] += toff[i];
            ooff[i + 1] += ooff[i];
        }
        par(s0, s1, [&](int i0, int i1) {
            for (int i = i0; i < i1; i++) {
                const int32_t* h = &hdr[(size_t)i * KL_HDR];
                kp_launch_result& r = results[i];
                r.status = h[0];
                r.failed_filter = h[1];
                r.capacity_type = h[2];
                r.n_types = h[3];
                r.n_options = h[5];
                for (int f = 0; f < KP_N_FILTERS; f++) r.rejected[f] = h[8 + f];
                r.type_offset = (int32_t)toff[i];
                r.override_offset = (int32_t)ooff[i];
                r.n_overrides = (int32_t)(ooff[i + 1] - ooff[i]);
                int64_t tp = toff[i], op = ooff[i];
                // kwok CreateFleet's lowest-price pick (kpsim.h kp_launch_result.fleet_pick): lo.MinBy over the overrides
                // in order; score = the spot price of (type, zone) for a spot fleet, else the type's on-demand price
                const bool spot = r.capacity_type == KP_CT_SPOT;
                int32_t pick = -1;
                double best = 0.0;
                for (int k = 0; k < r.n_types; k++, tp++) {
                    const int32_t t = tys[(size_t)i * M + k];
                    if (type_ids && tp < cap_type_ids) type_ids[tp] = t;
                    // override offerings of slot k: bit j = offering row off_begin[t] + j, ascending
                    for (uint64_t m = ov[(size_t)i * M + k]; m; m &= m - 1, op++) {
                        const int32_t row = c->l_off_begin[t] + __builtin_ctzll(m);
                        if (override_offerings && op < cap_overrides) override_offerings[op] = row;
                        double sc = DBL_MAX;
                        const int nO = (int)c->l_ct.size();
                        for (int f = c->l_off_begin[t]; f < c->l_off_begin[t + 1]; f++) {
                            if (spot ? (c->l_ct[f] == KP_CT_SPOT &&
                                        c->l_off_val[(size_t)KL_ROLE_ZONE * nO + f] == c->l_off_val[(size_t)KL_ROLE_ZONE * nO + row])
                                     : c->l_ct[f] == KP_CT_ON_DEMAND) {
                                sc = c->l_price[f];
                                break;
                            }
                        }
                        if (pick < 0 || best == 0.0 || (sc != 0.0 && sc < best)) {
                            pick = row;
                            best = sc;
                        }
                    }
                }
                r.fleet_pick = r.status == KP_OK ? pick : -1;
            }
        });
        ms_exp += ms_between(tx, clk::now());
        return hipSuccess;
    };
    c->pool.grow(nthr);
    for (int b = 0; b < nsub; b++) {
        const int s0 = sub_begin(b), s1 = sub_begin(b + 1), ns = s1 - s0;
        const int nt = std::max(1, std::min(nthr, (ns + 255) / 256));
        s = (b & 1) ? c->lstream2 : c->stream;
        const auto te0 = clk::now();
        for (auto& ch : chunks) {
            ch.keys.clear();
            ch.mins.clear();
            ch.words.clear();
        }
        if (!c->pool.run(nt, [&](int ti) {
                const int i0 = s0 + (int)((int64_t)ns * ti / nt), i1 = s0 + (int)((int64_t)ns * (ti + 1) / nt);
                for (int i = i0; i < i1; i++)
                    if (!encode_one(i, chunks[ti])) return;
            }))
            host_err = true;
        if (host_err) {
            hipStreamSynchronize(c->stream);  // no copy may still read the staging when the caller sees the error
            if (c->lstream2) hipStreamSynchronize(c->lstream2);
            return fail(c, KP_E_INVALID, "kp_launch_select: host error in a worker thread");
        }
        const auto te1 = clk::now();
        ms_enc += ms_between(te0, te1);
        // chunk tables concatenated straight into pinned staging, offsets rebased per chunk
        size_t nk = 0, nm = 0, nw = 0;
        for (int ti = 0; ti < nt; ti++) {
            if (chunks[ti].st != KP_OK) {
                hipStreamSynchronize(c->stream);  // no copy may still read the staging when the caller sees the error
                if (c->lstream2) hipStreamSynchronize(c->lstream2);
                return fail(c, chunks[ti].st, chunks[ti].msg);
            }
            nk += chunks[ti].keys.size();
            nm += chunks[ti].mins.size();
            nw += chunks[ti].words.size();
        }
        const int set = b & 1;
        HIPCHK(c->p_l_keys[set].ensure(std::max<size_t>(nk, 1)));
        HIPCHK(c->p_l_mins[set].ensure(std::max<size_t>(nm, 1)));
        HIPCHK(c->p_l_words[set].ensure(std::max<size_t>(nw, 1)));
        {
            size_t kb = 0, mb = 0, wbase = 0;
            for (int ti = 0; ti < nt; ti++) {
                Chunk& ch = chunks[ti];
                const int i0 = s0 + (int)((int64_t)ns * ti / nt), i1 = s0 + (int)((int64_t)ns * (ti + 1) / nt);
                for (int i = i0; i < i1; i++) {
                    KlReq& q = reqs[i];
                    q.key_off += (int)kb;
                    q.und_off += (int)kb;
                    q.min_off += (int)mb;
                    for (int r = 0; r < KL_ROLES; r++)
                        if (q.role[r].mode == KLR_CONSTRAINED) q.role[r].woff += (int)wbase;
                }
                KlKey* kd = c->p_l_keys[set].p + kb;
                for (size_t j = 0; j < ch.keys.size(); j++) {
                    kd[j] = ch.keys[j];
                    kd[j].woff += (int)wbase;  // undefined-key entries carry no bitset; their woff is never read
                }
                if (!ch.mins.empty()) memcpy(c->p_l_mins[set].p + mb, ch.mins.data(), ch.mins.size() * sizeof(KlMinKey));
                if (!ch.words.empty()) memcpy(c->p_l_words[set].p + wbase, ch.words.data(), ch.words.size() * sizeof(uint64_t));
                kb += ch.keys.size();
                mb += ch.mins.size();
                wbase += ch.words.size();
            }
        }
        KpLaunch g = g0;
        g.L = ns;
        if (ns > 0) {
            auto up = [&](auto& dbuf, const auto* src, size_t count) -> hipError_t {
                hipError_t e = dbuf.ensure(std::max<size_t>(count, 1));
                if (e != hipSuccess || count == 0) return e;
                return hipMemcpyAsync(dbuf.p, src, count * sizeof(*src), hipMemcpyHostToDevice, s);
            };
            HIPCHK(hipMemcpyAsync(c->d_l_req.p + s0, reqs + s0, (size_t)ns * sizeof(KlReq), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(c->d_l_rq.p + (size_t)s0 * R, rq + (size_t)s0 * R, (size_t)ns * R * sizeof(int64_t),
                                  hipMemcpyHostToDevice, s));
            HIPCHK(up(c->d_l_keys[set], c->p_l_keys[set].p, nk));
            HIPCHK(up(c->d_l_mins[set], c->p_l_mins[set].p, nm));
            HIPCHK(up(c->d_l_words[set], c->p_l_words[set].p, nw));
            g.req = c->d_l_req.p + s0;
            g.keys = c->d_l_keys[set].p;
            g.mins = c->d_l_mins[set].p;
            g.words = c->d_l_words[set].p;
            g.requests = c->d_l_rq.p + (size_t)s0 * R;
            g.out_hdr = c->d_l_hdr.p + (size_t)s0 * KL_HDR;
            g.out_types = c->d_l_types.p + (size_t)s0 * M;
            g.out_over = c->d_l_over.p + (size_t)s0 * M;
        }
        HIPCHK(hipEventRecord(c->lev[3 * b], s));
        if (ns > 0) HIPCHK(kp_launch_select_kernel(g, s));
        HIPCHK(hipEventRecord(c->lev[3 * b + 1], s));
        if (ns > 0) {
            HIPCHK(hipMemcpyAsync(c->p_l_hdr.p + (size_t)s0 * KL_HDR, g.out_hdr, (size_t)ns * KL_HDR * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(c->p_l_types.p + (size_t)s0 * M, g.out_types, (size_t)ns * M * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(c->p_l_over.p + (size_t)s0 * M, g.out_over, (size_t)ns * M * 8, hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipEventRecord(c->lev[3 * b + 2], s));
        ms_up += ms_between(te1, clk::now());
        if (b > 0) HIPCHK(expand(b - 1));
    }
    HIPCHK(expand(nsub - 1));
    if (host_err) return fail(c, KP_E_INVALID, "kp_launch_select: host error in a worker thread");
    const bool short_buf = (n > 0 && toff[n] > 0 && (!type_ids || toff[n] > cap_type_ids)) ||
                           (n > 0 && ooff[n] > 0 && (!override_offerings || ooff[n] > cap_overrides));
    c->launch_ms[0] = kms_sum;  // Σ kernel time over the sub-batches
    {
        std::sort(span, span + nsub);
        double busy = 0, hi = -1;
        for (int b = 0; b < nsub; b++) {
            const double lo = std::max<double>(span[b].first, hi);
            if (span[b].second > lo) busy += span[b].second - lo;
            hi = std::max<double>(hi, span[b].second);
        }
        c->launch_busy_ms = busy;
    }
    c->launch_ms[1] = ns_since(t0) / 1e6;
    c->launch_ms[2] = ms_enc;
    c->launch_ms[3] = ms_up;
    c->launch_ms[4] = ms_wait;
    c->launch_ms[5] = ms_exp;
    c->launch_nsub = nsub;
    if (short_buf) return fail(c, KP_E_BUFFER, "type_ids / override_offerings too small");
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

// instanceToNodeClaim (pkg/cloudprovider/cloudprovider.go:381-444) for an instance launched from catalog row
// type_index through offering row `offering` (its zone, capacity type and reservation are the instance's).
extern "C" kp_status kp_nodeclaim_labels(kp_ctx* ctx, int32_t type_index, int32_t offering, const char* zone_id,
                                         const char* nodepool, int32_t efa_enabled, char* buf, int64_t cap,
                                         int64_t* needed, int64_t* capacity, int64_t* allocatable) try {
    if (!ctx) return KP_E_INVALID;
    if (!ctx->have_catalog) return fail(ctx, KP_E_STATE, "kp_nodeclaim_labels before kp_catalog_upload");
    kp_ctx* c = ctx;
    const int T = c->T, O = (int)c->l_ct.size(), R = c->R;
    if (type_index < 0 || type_index >= T) return fail(c, KP_E_INVALID, "type_index out of range");
    if (offering < 0 || offering >= O) return fail(c, KP_E_INVALID, "offering out of range");
    if (c->off_type[offering] != type_index) return fail(c, KP_E_INVALID, "offering is not an offering of type_index");
    std::map<std::string, std::string> labels;
    // labels of the type's single-valued requirements, except the reservation keys (present for every capacity type)
    for (const auto& kv : c->type_single[type_index]) {
        if (kv.first == c->key_resvid || kv.first == c->key_resvtype) continue;
        const KeyDict& kd = c->cat.keys[kv.first];
        labels[kd.name] = kd.vals[kv.second];
    }
    auto role_val = [&](int role, int key) -> const std::string* {
        const int v = c->l_off_val[(size_t)role * O + offering];
        if (key < 0 || v < 0 || v >= (int)c->cat.keys[key].vals.size()) return nullptr;
        return &c->cat.keys[key].vals[v];
    };
    if (const std::string* z = role_val(KL_ROLE_ZONE, c->key_zone)) labels["topology.kubernetes.io/zone"] = *z;
    // zone-id: the EC2NodeClass subnet of the zone (the caller's), else the offering's own zone-id requirement
    if (zone_id && *zone_id) labels["topology.k8s.aws/zone-id"] = zone_id;
    else if (const std::string* zi = role_val(KL_ROLE_ZONEID, c->key_zoneid)) labels["topology.k8s.aws/zone-id"] = *zi;
    const int ct = c->l_ct[offering];
    labels["karpenter.sh/capacity-type"] = ct == KP_CT_SPOT ? "spot" : ct == KP_CT_RESERVED ? "reserved" : "on-demand";
    if (ct == KP_CT_RESERVED) {
        if (const std::string* r = role_val(KL_ROLE_RESVID, c->key_resvid)) labels["karpenter.k8s.aws/capacity-reservation-id"] = *r;
        if (const std::string* r = role_val(KL_ROLE_RESVTYPE, c->key_resvtype))
            labels["karpenter.k8s.aws/capacity-reservation-type"] = *r;
    }
    if (nodepool && *nodepool) labels["karpenter.sh/nodepool"] = nodepool;  // the instance's NodePool tag
    std::string out;
    for (auto& kv : labels) out += kv.first + "\t" + kv.second + "\n";
    if (needed) *needed = (int64_t)out.size() + 1;
    // Status.Capacity / Allocatable: non-zero quantities; EFA only when the launch requested EFA interfaces
    for (int r = 0; r < R; r++) {
        const bool efa = c->resource_names[r] == "vpc.amazonaws.com/efa";
        const int64_t cv = c->cap_rt[(size_t)r * T + type_index], av = c->alloc_rt[(size_t)r * T + type_index];
        const bool keep_c = cv != 0 && (!efa || efa_enabled), keep_a = av != 0 && (!efa || efa_enabled);
        if (capacity) capacity[r] = keep_c ? cv : 0;
        if (allocatable) allocatable[r] = keep_a ? av : 0;
    }
    if (!buf || cap < (int64_t)out.size() + 1) return fail(c, KP_E_BUFFER, "label buffer too small");
    memcpy(buf, out.c_str(), out.size() + 1);
    return KP_OK;
} catch (const std::exception& e) {
    return fail(ctx, KP_E_INVALID, e.what());
}

extern "C" kp_status kp_launch_stats(kp_ctx* ctx, double* ms, int32_t n) {
    if (!ctx || !ms) return KP_E_INVALID;
    for (int i = 0; i < n && i < 6; i++) ms[i] = ctx->launch_ms[i];
    if (n > 6) ms[6] = ctx->launch_nsub;
    if (n > 7) ms[7] = ctx->launch_busy_ms;
    return KP_OK;
}
