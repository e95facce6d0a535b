// ORACLE — test infrastructure only (see oracle/README.md). Never linked into libkpsim.
//
// CPU restatement of the [core] label-requirement algebra (sigs.k8s.io/karpenter@v1.6.1-0.20250908174930,
// pkg/scheduling/requirement.go + requirements.go; not vendored in the reference, semantics recalled and
// cross-checked against in-tree call sites: pkg/providers/instancetype/types.go:151,181-234,
// pkg/providers/instance/filter/filter.go:53, offering.go:141-151 and the KATs in tests/golden/kats.json).
//
// Strings are interned per key (Go uses sets.Set[string]; set semantics are identical).
#pragma once
#include <algorithm>
#include <cstdint>
#include <climits>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace orc {

enum Op { OP_IN = 0, OP_NOT_IN = 1, OP_EXISTS = 2, OP_DNE = 3, OP_GT = 4, OP_LT = 5 };

// Go strconv.Atoi on a 64-bit platform: optional sign, decimal digits, no spaces, range-checked.
inline bool go_atoi(const std::string& s, int64_t& out) {
    size_t i = 0;
    bool neg = false;
    if (s.empty()) return false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
    }
    if (i >= s.size()) return false;
    unsigned __int128 v = 0;
    for (; i < s.size(); i++) {
        char c = s[i];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (unsigned)(c - '0');
        if (v > (unsigned __int128)1 << 63) return false;
    }
    if (!neg && v > (unsigned __int128)INT64_MAX) return false;
    out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
    return true;
}

// karpv1.WellKnownLabels ([core] pkg/apis/v1/labels.go) + the AWS additions registered at
// pkg/apis/v1/labels.go:31-57.  Used as AllowUndefinedWellKnownLabels.
inline bool is_well_known_label(const std::string& k) {
    static const char* const wk[] = {
        "karpenter.sh/nodepool", "topology.kubernetes.io/zone", "topology.kubernetes.io/region",
        "node.kubernetes.io/instance-type", "kubernetes.io/arch", "kubernetes.io/os", "karpenter.sh/capacity-type",
        "node.kubernetes.io/windows-build",
        // AWS (labels.go:31-57)
        "karpenter.k8s.aws/capacity-reservation-id", "karpenter.k8s.aws/capacity-reservation-type",
        "karpenter.k8s.aws/instance-hypervisor", "karpenter.k8s.aws/instance-encryption-in-transit-supported",
        "karpenter.k8s.aws/instance-category", "karpenter.k8s.aws/instance-capacity-flex",
        "karpenter.k8s.aws/instance-family", "karpenter.k8s.aws/instance-generation",
        "karpenter.k8s.aws/instance-size", "karpenter.k8s.aws/instance-local-nvme", "karpenter.k8s.aws/instance-cpu",
        "karpenter.k8s.aws/instance-cpu-manufacturer", "karpenter.k8s.aws/instance-cpu-sustained-clock-speed-mhz",
        "karpenter.k8s.aws/instance-memory", "karpenter.k8s.aws/instance-ebs-bandwidth",
        "karpenter.k8s.aws/instance-network-bandwidth", "karpenter.k8s.aws/instance-gpu-name",
        "karpenter.k8s.aws/instance-gpu-manufacturer", "karpenter.k8s.aws/instance-gpu-count",
        "karpenter.k8s.aws/instance-gpu-memory", "karpenter.k8s.aws/instance-accelerator-name",
        "karpenter.k8s.aws/instance-accelerator-manufacturer", "karpenter.k8s.aws/instance-accelerator-count",
        "topology.k8s.aws/zone-id",
    };
    for (auto* w : wk)
        if (k == w) return true;
    return false;
}

// karpv1.NormalizedLabels (+ "topology.ebs.csi.aws.com/zone", pkg/operator/operator.go:71).
inline std::string normalize_label(const std::string& k) {
    if (k == "failure-domain.beta.kubernetes.io/zone") return "topology.kubernetes.io/zone";
    if (k == "failure-domain.beta.kubernetes.io/region") return "topology.kubernetes.io/region";
    if (k == "beta.kubernetes.io/arch") return "kubernetes.io/arch";
    if (k == "beta.kubernetes.io/os") return "kubernetes.io/os";
    if (k == "beta.kubernetes.io/instance-type") return "node.kubernetes.io/instance-type";
    if (k == "topology.ebs.csi.aws.com/zone") return "topology.kubernetes.io/zone";
    return k;
}

// Interning dictionary shared by a solve.
struct Dict {
    std::vector<uint8_t> well_known;  // per key id
    std::unordered_map<std::string, int> key_id;
    std::vector<std::string> keys;
    std::vector<std::unordered_map<std::string, int>> val_id;  // per key
    std::vector<std::vector<std::string>> vals;
    std::vector<std::vector<uint8_t>> val_isint;
    std::vector<std::vector<int64_t>> val_int;

    int key(const std::string& k) {
        auto it = key_id.find(k);
        if (it != key_id.end()) return it->second;
        int id = (int)keys.size();
        key_id.emplace(k, id);
        keys.push_back(k);
        well_known.push_back(is_well_known_label(k) ? 1 : 0);
        val_id.emplace_back();
        vals.emplace_back();
        val_isint.emplace_back();
        val_int.emplace_back();
        return id;
    }
    int value(int k, const std::string& v) {
        auto& m = val_id[k];
        auto it = m.find(v);
        if (it != m.end()) return it->second;
        int id = (int)vals[k].size();
        m.emplace(v, id);
        vals[k].push_back(v);
        int64_t x = 0;
        bool ok = go_atoi(v, x);
        val_isint[k].push_back(ok ? 1 : 0);
        val_int[k].push_back(x);
        return id;
    }
};

// scheduling.Requirement
struct Req {
    int key = -1;
    bool complement = false;
    std::vector<int> values;  // sorted, unique value ids
    bool has_gt = false, has_lt = false;
    int64_t gt = 0, lt = 0;
    bool has_min = false;
    int min_values = 0;

    // Len(): complement → MaxInt64 − |values|, else |values|
    int64_t Len() const { return complement ? (INT64_MAX - (int64_t)values.size()) : (int64_t)values.size(); }
    // Operator()
    Op Operator() const {
        if (complement) return Len() < INT64_MAX ? OP_NOT_IN : OP_EXISTS;
        return Len() > 0 ? OP_IN : OP_DNE;
    }
    bool has_value(int v) const { return std::binary_search(values.begin(), values.end(), v); }
};

// withinIntPtrs(value, gt, lt).  Negative value ids are NodeClaim hostname placeholders
// ("hostname-placeholder-NNNN", never an integer).
inline bool within(const Dict& D, int key, int v, bool has_gt, int64_t gt, bool has_lt, int64_t lt) {
    if (!has_gt && !has_lt) return true;
    if (v < 0 || !D.val_isint[key][v]) return false;
    int64_t x = D.val_int[key][v];
    if (has_gt && gt >= x) return false;
    if (has_lt && lt <= x) return false;
    return true;
}

// Requirement.Has(value)
inline bool req_has(const Dict& D, const Req& r, int v) {
    bool in = r.has_value(v);
    if (r.complement) return !in && within(D, r.key, v, r.has_gt, r.gt, r.has_lt, r.lt);
    return in && within(D, r.key, v, r.has_gt, r.gt, r.has_lt, r.lt);
}

// NewRequirementWithFlexibility(key, op, minValues, values...)
inline Req new_req(Dict& D, int key, Op op, const std::vector<std::string>& values, bool has_min, int min_values) {
    Req r;
    r.key = key;
    r.complement = true;
    r.has_min = has_min;
    r.min_values = min_values;
    if (op == OP_IN || op == OP_DNE) r.complement = false;
    if (op == OP_IN || op == OP_NOT_IN) {
        for (auto& s : values) r.values.push_back(D.value(key, s));
        std::sort(r.values.begin(), r.values.end());
        r.values.erase(std::unique(r.values.begin(), r.values.end()), r.values.end());
    }
    if (op == OP_GT) {
        int64_t x = 0;
        go_atoi(values.empty() ? std::string() : values[0], x);  // prevalidated by the API
        r.has_gt = true;
        r.gt = x;
    }
    if (op == OP_LT) {
        int64_t x = 0;
        go_atoi(values.empty() ? std::string() : values[0], x);
        r.has_lt = true;
        r.lt = x;
    }
    return r;
}

// Requirement.Intersection(requirement)
inline Req req_intersection(const Dict& D, const Req& r, const Req& q) {
    Req o;
    o.key = r.key;
    o.complement = r.complement && q.complement;
    // boundaries
    o.has_gt = r.has_gt || q.has_gt;
    o.gt = r.has_gt && q.has_gt ? std::max(r.gt, q.gt) : (r.has_gt ? r.gt : q.gt);
    o.has_lt = r.has_lt || q.has_lt;
    o.lt = r.has_lt && q.has_lt ? std::min(r.lt, q.lt) : (r.has_lt ? r.lt : q.lt);
    o.has_min = r.has_min || q.has_min;
    o.min_values = r.has_min && q.has_min ? std::max(r.min_values, q.min_values) : (r.has_min ? r.min_values : q.min_values);
    if (o.has_gt && o.has_lt && o.gt >= o.lt) {
        Req d;
        d.key = r.key;
        d.complement = false;  // DoesNotExist
        d.has_min = o.has_min;
        d.min_values = o.min_values;
        return d;
    }
    std::vector<int> vals;
    if (r.complement && q.complement) {
        std::set_union(r.values.begin(), r.values.end(), q.values.begin(), q.values.end(), std::back_inserter(vals));
    } else if (r.complement && !q.complement) {
        std::set_difference(q.values.begin(), q.values.end(), r.values.begin(), r.values.end(), std::back_inserter(vals));
    } else if (!r.complement && q.complement) {
        std::set_difference(r.values.begin(), r.values.end(), q.values.begin(), q.values.end(), std::back_inserter(vals));
    } else {
        std::set_intersection(r.values.begin(), r.values.end(), q.values.begin(), q.values.end(), std::back_inserter(vals));
    }
    for (int v : vals)
        if (within(D, r.key, v, o.has_gt, o.gt, o.has_lt, o.lt)) o.values.push_back(v);
    if (!o.complement) {  // remove boundaries for concrete sets
        o.has_gt = o.has_lt = false;
        o.gt = o.lt = 0;
    }
    return o;
}

// scheduling.Requirements (map[string]*Requirement) as a key-ordered map.
struct Reqs {
    std::map<int, Req> m;
    bool has(int k) const { return m.count(k) != 0; }
    // Get(key): undefined keys are treated as Exists
    Req get(int k) const {
        auto it = m.find(k);
        if (it != m.end()) return it->second;
        Req r;
        r.key = k;
        r.complement = true;
        return r;
    }
    // Add(requirements...): intersect with existing
    void add(const Dict& D, const Req& q) {
        auto it = m.find(q.key);
        if (it != m.end()) {
            it->second = req_intersection(D, q, it->second);
        } else {
            m.emplace(q.key, q);
        }
    }
    void add_all(const Dict& D, const Reqs& o) {
        for (auto& kv : o.m) add(D, kv.second);
    }
    bool has_min_values() const {
        for (auto& kv : m)
            if (kv.second.has_min) return true;
        return false;
    }
};

// Requirements.Intersects(requirements) == nil
inline bool reqs_intersects(const Dict& D, const Reqs& r, const Reqs& q) {
    // iterate the smaller map
    const Reqs& a = r.m.size() <= q.m.size() ? r : q;
    const Reqs& b = r.m.size() <= q.m.size() ? q : r;
    for (auto& kv : a.m) {
        auto it = b.m.find(kv.first);
        if (it == b.m.end()) continue;
        const Req& existing = (&a == &r) ? kv.second : it->second;
        const Req& incoming = (&a == &r) ? it->second : kv.second;
        Req x = req_intersection(D, existing, incoming);
        if (x.Len() == 0) {
            Op io = incoming.Operator();
            if (io == OP_NOT_IN || io == OP_DNE) {
                Op eo = existing.Operator();
                if (eo == OP_NOT_IN || eo == OP_DNE) continue;
            }
            return false;
        }
    }
    return true;
}

// Requirements.Compatible(requirements, opts) == nil.  allow_wk = AllowUndefinedWellKnownLabels.
inline bool reqs_compatible(const Dict& D, const Reqs& r, const Reqs& q, bool allow_wk) {
    for (auto& kv : q.m) {
        if (r.has(kv.first)) continue;
        Op o = kv.second.Operator();
        if (o == OP_NOT_IN || o == OP_DNE) continue;
        if (allow_wk && D.well_known[kv.first]) continue;
        return false;
    }
    return reqs_intersects(D, r, q);
}

}  // namespace orc
