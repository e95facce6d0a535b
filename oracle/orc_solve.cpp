// ORACLE — test infrastructure only (see oracle/README.md). Never linked into libkpsim; only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg load liboracle.so, and only as the checker.
//
// CPU restatement of the reference's provisioning scheduling simulation:
//   [core] pkg/controllers/provisioning/scheduling/scheduler.go  NewScheduler / Solve / add
//          (sort.Slice(newNodeClaims, by len(Pods)) before every in-flight attempt, templates in weight order,
//           filterByRemainingResources / subtractMax NodePool limits)
//   [core] .../scheduling/queue.go          NewQueue (byCPUAndMemoryDescending), Pop, Push
//   [core] .../scheduling/nodeclaim.go      NewNodeClaim, Add, FinalizeScheduling,
//                                            filterInstanceTypesByRequirements (compatible, fits, hasOffering, minValues)
//   [core] .../scheduling/existingnode.go   ExistingNode.Add
//   [core] pkg/cloudprovider/types.go       InstanceTypes.OrderByPrice / Truncate / SatisfiesMinValues,
//                                            Offerings.Available / Compatible / Cheapest
//   [core] pkg/utils/resources              Fits, Merge, MaxResources
// Core is sigs.k8s.io/karpenter v1.6.1-0.20250908174930-91341612ebc6 (reference go.mod:49), not vendored:
// semantics are recalled and pinned by the KATs from the reference's own suites
// (tests/golden/kats.json; pkg/providers/instancetype/suite_test.go:395-995).  In-tree inputs follow
// pkg/providers/instancetype/offering/offering.go:103-196 (offering requirements) and
// pkg/providers/instance/instance.go:62,293 (maxInstanceTypes = 60, Truncate).
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/kpsim.h"
#include "gosort.h"
#include "orc_api.h"
#include "orc_req.h"

namespace orc {

struct Offering {
    Reqs reqs;
    double price = 0;
    bool available = false;
};

struct InstanceType {
    std::string name;
    Reqs reqs;
    std::vector<int64_t> cap, alloc;
    std::vector<Offering> offerings;
};

struct Taint {
    std::string key, value, effect;
};
struct Toleration {
    std::string key;
    int op = 0;
    std::string value, effect;
};

// k8s.io/api/core/v1 Toleration.ToleratesTaint
static bool tolerates_taint(const Toleration& t, const Taint& taint) {
    if (!t.effect.empty() && t.effect != taint.effect) return false;
    if (!t.key.empty() && t.key != taint.key) return false;
    if (t.op == KP_TOL_EXISTS) return true;
    return t.value == taint.value;
}
// [core] scheduling.Taints.ToleratesPod: every taint must be tolerated by some toleration
static bool tolerates_all(const std::vector<Taint>& taints, const std::vector<Toleration>& tols) {
    for (auto& taint : taints) {
        bool ok = false;
        for (auto& t : tols) ok = ok || tolerates_taint(t, taint);
        if (!ok) return false;
    }
    return true;
}

// [core] resources.Fits(candidate, total)
static bool fits(const std::vector<int64_t>& candidate, const std::vector<int64_t>& total) {
    for (int64_t q : total)
        if (q < 0) return false;
    for (size_t r = 0; r < candidate.size(); r++)
        if (candidate[r] > total[r]) return false;
    return true;
}

struct PodClass {
    Reqs reqs;
    std::vector<Toleration> tols;
};
struct Pod {
    int cls = 0;
    std::vector<int64_t> req;
    int64_t ts = 0;
    std::string uid;
};

struct Template {
    int np_index = 0;
    std::string name;
    int weight = 0;
    Reqs reqs;
    std::vector<Taint> taints;
    std::vector<int64_t> daemon;
    std::vector<uint8_t> limit_set;
    std::vector<int64_t> remaining;
    std::vector<int> options;  // InstanceTypeOptions (catalog rows, order = GetInstanceTypes order)
};

struct NodeClaim {
    int id = 0;
    int tmpl = 0;
    Reqs reqs;
    std::vector<int> options;
    std::vector<int64_t> requests;
    std::vector<int> pods;
    bool valid = true;
    std::vector<int> truncated;
};

struct ExistingNode {
    Reqs reqs;
    std::vector<Taint> taints;
    std::vector<int64_t> available, requests;
};

struct Result {
    std::vector<NodeClaim> ncs;  // creation order
    Dict D;
};

struct Solver {
    Dict& D;
    int R = 0;
    std::vector<InstanceType> own_types;
    const std::vector<InstanceType>* tp = &own_types;  // catalog rows (shared by consolidation probes)
    std::vector<Template> tmpls;
    std::vector<PodClass> own_classes;
    const std::vector<PodClass>* cp = &own_classes;
    std::vector<Pod> own_pods;
    const std::vector<Pod>* pp = &own_pods;
    std::vector<ExistingNode> own_existing;
    const std::vector<ExistingNode>* ex_base = &own_existing;  // state nodes (shared by consolidation probes)
    std::vector<int> ex_idx;                                 // existing nodes of this simulation, in order
    std::unordered_map<int, ExistingNode> ex_mod;            // copy-on-write: nodes that received pods
    std::vector<int> plist;           // pods of this simulation (indices into *pp); all per-pod state is by position
    std::vector<NodeClaim> ncs;       // creation order; nc.pods holds positions in plist
    std::vector<int> newNodeClaims;   // s.newNodeClaims slice (indices into ncs)
    std::vector<int> pod_result, pod_order;  // by position in plist
    int placements = 0;
    int hostname_key = -1;
    Req host_req;                     // hostname In [placeholder] of a new NodeClaim (no pod can select it)
    kp_solve_stats stats{};

    explicit Solver(Dict& d) : D(d) {}
    const InstanceType& ty(int t) const { return (*tp)[t]; }
    const Pod& pod_at(int li) const { return (*pp)[plist[li]]; }
    const PodClass& cls_of(int li) const { return (*cp)[pod_at(li).cls]; }

    // compatible(it, reqs) = it.Requirements.Intersects(reqs) == nil
    bool compatible(const InstanceType& it, const Reqs& reqs) const { return reqs_intersects(D, it.reqs, reqs); }
    bool has_offering(const InstanceType& it, const Reqs& reqs) const {
        for (auto& o : it.offerings)
            if (o.available && reqs_compatible(D, reqs, o.reqs, true)) return true;
        return false;
    }
    // InstanceTypes.SatisfiesMinValues(requirements): minNeededInstanceTypes (the shortest prefix that satisfies every
    // minValues key) and whether the whole list satisfies them.
    bool satisfies_min_values(const std::vector<int>& its, const Reqs& reqs, int* min_needed = nullptr) const {
        if (min_needed) *min_needed = 0;
        if (!reqs.has_min_values()) return true;
        std::vector<std::pair<int, std::vector<int>>> seen;  // (key, sorted distinct values so far)
        for (auto& kv : reqs.m)
            if (kv.second.has_min) seen.push_back({kv.first, {}});
        for (size_t i = 0; i < its.size(); i++) {
            bool ok = true;
            for (auto& sk : seen) {
                Req r = ty(its[i]).reqs.get(sk.first);
                for (int v : r.values) sk.second.push_back(v);
                std::sort(sk.second.begin(), sk.second.end());
                sk.second.erase(std::unique(sk.second.begin(), sk.second.end()), sk.second.end());
                if ((int)sk.second.size() < reqs.m.at(sk.first).min_values) ok = false;
            }
            if (ok) {
                if (min_needed) *min_needed = (int)i + 1;
                return true;
            }
        }
        if (min_needed) *min_needed = (int)its.size();
        for (auto& sk : seen)
            if ((int)sk.second.size() < reqs.m.at(sk.first).min_values) return false;
        return true;
    }
    // filterInstanceTypesByRequirements (MIN_VALUES_POLICY=Strict)
    std::vector<int> filter(const std::vector<int>& its, const Reqs& reqs, const std::vector<int64_t>& total) const {
        std::vector<int> out;
        for (int t : its) {
            const InstanceType& it = ty(t);
            if (compatible(it, reqs) && fits(total, it.alloc) && has_offering(it, reqs)) out.push_back(t);
        }
        if (reqs.has_min_values() && !satisfies_min_values(out, reqs)) out.clear();
        return out;
    }

    bool nodeclaim_add(NodeClaim& nc, int li) {
        const Pod& pod = pod_at(li);
        const PodClass& pc = cls_of(li);
        const Template& tm = tmpls[nc.tmpl];
        if (!tolerates_all(tm.taints, pc.tols)) return false;
        Reqs r = nc.reqs;
        if (!reqs_compatible(D, r, pc.reqs, true)) return false;
        r.add_all(D, pc.reqs);
        // topology.AddRequirements: no topology groups in this build's inputs → the requirements themselves;
        // Compatible(r, r) always holds and Add(r) is idempotent.
        std::vector<int64_t> requests(R);
        for (int k = 0; k < R; k++) requests[k] = nc.requests[k] + pod.req[k];
        std::vector<int> remaining = filter(nc.options, r, requests);
        if (remaining.empty()) return false;
        nc.pods.push_back(li);
        nc.options.swap(remaining);
        nc.requests.swap(requests);
        nc.reqs = std::move(r);
        return true;
    }

    // ExistingNode.Add: Taints.ToleratesPod, Fits(requests + pod, available), Compatible (no undefined-label
    // allowance), then requirements.Add.  On success `out` is the updated node.
    bool existing_try(const ExistingNode& n, int li, ExistingNode& out) {
        const Pod& pod = pod_at(li);
        const PodClass& pc = cls_of(li);
        if (!tolerates_all(n.taints, pc.tols)) return false;
        std::vector<int64_t> requests(R);
        for (int k = 0; k < R; k++) requests[k] = n.requests[k] + pod.req[k];
        if (!fits(requests, n.available)) return false;
        Reqs r = n.reqs;
        if (!reqs_compatible(D, r, pc.reqs, false)) return false;
        r.add_all(D, pc.reqs);
        out.taints = n.taints;
        out.available = n.available;
        out.requests.swap(requests);
        out.reqs = std::move(r);
        return true;
    }

    // sort.Slice(s.newNodeClaims, func(a, b int) bool { return len(a.Pods) < len(b.Pods) })
    struct SliceAdaptor {
        Solver* s;
        int size() const { return (int)s->newNodeClaims.size(); }
        bool less(int i, int j) const {
            return s->ncs[s->newNodeClaims[i]].pods.size() < s->ncs[s->newNodeClaims[j]].pods.size();
        }
        void swap(int i, int j) { std::swap(s->newNodeClaims[i], s->newNodeClaims[j]); }
    };

    bool add(int li) {
        for (int j : ex_idx) {
            stats.existing_evals++;
            auto it = ex_mod.find(j);
            const ExistingNode& n = it != ex_mod.end() ? it->second : (*ex_base)[j];
            ExistingNode upd;
            if (existing_try(n, li, upd)) {
                ex_mod[j] = std::move(upd);
                pod_result[li] = KP_POD_EXISTING(j);
                return true;
            }
        }
        SliceAdaptor sa{this};
        go_sort_slice(sa);
        stats.nodeclaim_candidates_scanned += (int64_t)newNodeClaims.size();
        for (int idx : newNodeClaims) {
            stats.nodeclaim_evals++;
            if (nodeclaim_add(ncs[idx], li)) {
                pod_result[li] = idx;
                return true;
            }
        }
        for (size_t ti = 0; ti < tmpls.size(); ti++) {
            Template& tm = tmpls[ti];
            // filterByRemainingResources(its, remaining)
            std::vector<int> its;
            for (int t : tm.options) {
                bool viable = true;
                for (int k = 0; k < R; k++)
                    if (tm.limit_set[k] && ty(t).cap[k] > tm.remaining[k]) viable = false;
                if (viable) its.push_back(t);
            }
            if (its.empty()) continue;
            // NewNodeClaim
            NodeClaim nc;
            nc.id = (int)ncs.size();
            nc.tmpl = (int)ti;
            nc.reqs = tm.reqs;
            nc.reqs.add(D, host_req);
            nc.options = its;
            nc.requests = tm.daemon;
            stats.template_evals++;
            if (!nodeclaim_add(nc, li)) continue;
            // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
            for (int k = 0; k < R; k++) {
                if (!tm.limit_set[k]) continue;
                int64_t mx = 0;
                bool first = true;
                for (int t : nc.options) {
                    if (first || ty(t).cap[k] > mx) mx = ty(t).cap[k];
                    first = false;
                }
                tm.remaining[k] -= mx;
            }
            ncs.push_back(std::move(nc));
            newNodeClaims.push_back((int)ncs.size() - 1);
            pod_result[li] = (int)ncs.size() - 1;
            return true;
        }
        return false;
    }

    void solve() {
        // NewQueue: sort.Slice(pods, byCPUAndMemoryDescending) — a total order (Kubernetes UIDs are unique).  Inputs
        // without UIDs (kp_pods_view.uids NULL) keep their input order on ties, as the device's stable radix passes do.
        const int n = (int)plist.size();
        std::vector<int> order(n);
        for (int i = 0; i < n; i++) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
            const Pod& l = pod_at(a);
            const Pod& r = pod_at(b);
            if (l.req[cpu_axis] != r.req[cpu_axis]) return l.req[cpu_axis] > r.req[cpu_axis];
            if (l.req[mem_axis] != r.req[mem_axis]) return l.req[mem_axis] > r.req[mem_axis];
            if (l.ts != r.ts) return l.ts < r.ts;
            return l.uid < r.uid;
        });
        std::deque<int> q(order.begin(), order.end());
        std::unordered_map<int, int> lastLen;
        pod_result.assign(n, KP_POD_UNSCHEDULABLE);
        pod_order.assign(n, -1);
        for (;;) {
            if (q.empty()) break;
            int li = q.front();
            auto it = lastLen.find(li);
            if (it != lastLen.end() && it->second == (int)q.size()) break;
            q.pop_front();
            stats.pods_popped++;
            if (add(li)) {
                pod_order[li] = placements++;
                continue;
            }
            // preferences.Relax: no preferred terms in this build's inputs → never relaxed
            q.push_back(li);
            lastLen[li] = (int)q.size();
        }
    }

    // Cheapest available offering compatible with reqs (OrderByPrice key); MaxFloat64 when none.
    double cheapest(int t, const Reqs& reqs) const {
        double price = DBL_MAX;
        bool any = false;
        for (auto& o : ty(t).offerings) {
            if (!o.available || !reqs_compatible(D, reqs, o.reqs, true)) continue;
            if (!any || o.price < price) price = o.price;
            any = true;
        }
        return any ? price : DBL_MAX;
    }

    // Solve's FinalizeScheduling + Results.TruncateInstanceTypes(maxInstanceTypes): hostname removed,
    // InstanceTypes.Truncate = OrderByPrice(reqs) then the first max types, SatisfiesMinValues on the kept list
    // (a NodeClaim that fails it is dropped and its pods get errors).
    void finalize(int max_types) {
        for (auto& nc : ncs) {
            nc.reqs.m.erase(hostname_key);
            std::vector<std::pair<double, int>> keyed;
            for (int t : nc.options) keyed.push_back({cheapest(t, nc.reqs), t});
            std::sort(keyed.begin(), keyed.end(), [&](const std::pair<double, int>& a, const std::pair<double, int>& b) {
                if (a.first == b.first) return ty(a.second).name < ty(b.second).name;
                return a.first < b.first;
            });
            std::vector<int> tr;
            for (auto& kv : keyed) tr.push_back(kv.second);
            if (max_types > 0 && (int)tr.size() > max_types) tr.resize(max_types);
            if (nc.reqs.has_min_values() && !satisfies_min_values(tr, nc.reqs)) {
                nc.valid = false;
                for (int li : nc.pods) {
                    pod_result[li] = KP_POD_UNSCHEDULABLE;
                    pod_order[li] = -1;
                }
            }
            nc.truncated = tr;
        }
    }
    int cpu_axis = 0, mem_axis = 1;
};

static std::vector<std::string> strs(const char* const* v, int n) {
    std::vector<std::string> o;
    for (int i = 0; i < n; i++) o.emplace_back(v[i] ? v[i] : "");
    return o;
}

static bool build_reqs(Dict& D, const kp_requirement* rs, int n, Reqs& out) {
    for (int i = 0; i < n; i++) {
        const kp_requirement& r = rs[i];
        if (!r.key || r.op < 0 || r.op > 5) return false;
        int k = D.key(normalize_label(r.key));
        out.add(D, new_req(D, k, (Op)r.op, strs(r.values, r.n_values), r.min_values >= 0, r.min_values));
    }
    return true;
}

}  // namespace orc

using namespace orc;

struct orc_result {
    std::vector<NodeClaim> ncs;
    Dict D;
};

// Input views → NewScheduler state (catalog rows, classes, pods, NodeClaimTemplates in weight order, existing nodes).
static kp_status parse_into(Solver& s, const kp_catalog_view* cat, const kp_solve_input* in) {
    Dict& D = s.D;
    const int T = cat->n_types, R = cat->n_resources;
    s.R = R;
    s.cpu_axis = s.mem_axis = -1;
    for (int r = 0; r < R; r++) {
        if (!strcmp(cat->resource_names[r], "cpu")) s.cpu_axis = r;
        if (!strcmp(cat->resource_names[r], "memory")) s.mem_axis = r;
    }
    if (s.cpu_axis < 0 || s.mem_axis < 0) return KP_E_INVALID;
    s.hostname_key = D.key("kubernetes.io/hostname");
    s.host_req = new_req(D, s.hostname_key, OP_IN, {"hostname-placeholder"}, false, 0);
    // catalog → []*cloudprovider.InstanceType
    s.own_types.resize(T);
    for (int t = 0; t < T; t++) {
        InstanceType& it = s.own_types[t];
        it.name = cat->type_names[t];
        it.cap.assign(cat->capacity + (size_t)t * R, cat->capacity + (size_t)(t + 1) * R);
        it.alloc.assign(cat->allocatable + (size_t)t * R, cat->allocatable + (size_t)(t + 1) * R);
        for (int k = 0; k < cat->n_label_keys; k++) {
            int st = cat->label_state[(size_t)t * cat->n_label_keys + k];
            if (st == KP_LABEL_ABSENT) continue;
            int key = D.key(normalize_label(cat->label_keys[k]));
            if (st == KP_LABEL_DOES_NOT_EXIST) {
                it.reqs.add(D, new_req(D, key, OP_DNE, {}, false, 0));
            } else {
                int o0 = cat->label_offsets[(size_t)t * cat->n_label_keys + k];
                int o1 = cat->label_offsets[(size_t)t * cat->n_label_keys + k + 1];
                it.reqs.add(D, new_req(D, key, OP_IN, strs(cat->label_values + o0, o1 - o0), false, 0));
            }
        }
    }
    for (int o = 0; o < cat->n_offerings; o++) {
        int t = cat->offering_type[o];
        if (t < 0 || t >= T) return KP_E_INVALID;
        Offering of;
        of.price = cat->offering_price[o];
        of.available = cat->offering_available[o] != 0;
        for (int k = 0; k < cat->n_offering_keys; k++) {
            int st = cat->offering_label_state[(size_t)o * cat->n_offering_keys + k];
            if (st == KP_LABEL_ABSENT) continue;
            int key = D.key(normalize_label(cat->offering_keys[k]));
            if (st == KP_LABEL_DOES_NOT_EXIST)
                of.reqs.add(D, new_req(D, key, OP_DNE, {}, false, 0));
            else
                of.reqs.add(D, new_req(D, key, OP_IN, {cat->offering_label_values[(size_t)o * cat->n_offering_keys + k]}, false, 0));
        }
        s.own_types[t].offerings.push_back(std::move(of));
    }
    // pod classes
    s.own_classes.resize(in->n_classes);
    for (int c = 0; c < in->n_classes; c++) {
        const kp_pod_class& pc = in->classes[c];
        if (!build_reqs(D, pc.requirements, pc.n_requirements, s.own_classes[c].reqs)) return KP_E_INVALID;
        for (int i = 0; i < pc.n_tolerations; i++) {
            Toleration t;
            t.key = pc.tolerations[i].key ? pc.tolerations[i].key : "";
            t.op = pc.tolerations[i].op;
            t.value = pc.tolerations[i].value ? pc.tolerations[i].value : "";
            t.effect = pc.tolerations[i].effect ? pc.tolerations[i].effect : "";
            s.own_classes[c].tols.push_back(t);
        }
    }
    // pods
    const kp_pods_view& pv = in->pods;
    s.own_pods.resize(pv.n_pods);
    for (int p = 0; p < pv.n_pods; p++) {
        Pod& pod = s.own_pods[p];
        pod.cls = pv.class_id[p];
        if (pod.cls < 0 || pod.cls >= in->n_classes) return KP_E_INVALID;
        pod.req.assign(pv.requests + (size_t)p * R, pv.requests + (size_t)(p + 1) * R);
        pod.ts = pv.creation_ns ? pv.creation_ns[p] : 0;
        pod.uid = pv.uids && pv.uids[p] ? pv.uids[p] : "";
    }
    // NodePools → NodeClaimTemplates, OrderByWeight (weight desc, name asc)
    std::vector<int> npo(in->n_nodepools);
    for (int i = 0; i < in->n_nodepools; i++) npo[i] = i;
    std::sort(npo.begin(), npo.end(), [&](int a, int b) {
        const kp_nodepool& x = in->nodepools[a];
        const kp_nodepool& y = in->nodepools[b];
        if (x.weight != y.weight) return x.weight > y.weight;
        return strcmp(x.name, y.name) < 0;
    });
    for (int i : npo) {
        const kp_nodepool& np = in->nodepools[i];
        Template tm;
        tm.np_index = i;
        tm.name = np.name;
        tm.weight = np.weight;
        if (!build_reqs(D, np.requirements, np.n_requirements, tm.reqs)) return KP_E_INVALID;
        for (int j = 0; j < np.n_taints; j++)
            tm.taints.push_back({np.taints[j].key ? np.taints[j].key : "", np.taints[j].value ? np.taints[j].value : "",
                                 np.taints[j].effect ? np.taints[j].effect : ""});
        tm.daemon.assign(R, 0);
        if (np.daemon_overhead) tm.daemon.assign(np.daemon_overhead, np.daemon_overhead + R);
        tm.limit_set.assign(R, 0);
        tm.remaining.assign(R, 0);
        if (np.limit_set) {
            tm.limit_set.assign(np.limit_set, np.limit_set + R);
            tm.remaining.assign(np.limit_remaining, np.limit_remaining + R);
        }
        std::vector<int> rows;
        if (np.n_types < 0) {
            for (int t = 0; t < T; t++) rows.push_back(t);
        } else {
            for (int j = 0; j < np.n_types; j++) rows.push_back(np.type_index[j]);
        }
        // NewScheduler: nct.InstanceTypeOptions = filterInstanceTypesByRequirements(its, nct.Requirements, {}, {}, {})
        std::vector<int64_t> zero(R, 0);
        // Fits({}, alloc) only rejects negative allocatable; emulate with an all-zero request
        tm.options = s.filter(rows, tm.reqs, zero);
        if (tm.options.empty()) continue;  // "skipping, nodepool requirements filtered out all instance types"
        s.tmpls.push_back(std::move(tm));
    }
    // existing nodes
    for (int j = 0; j < in->n_existing; j++) {
        const kp_existing_node& en = in->existing[j];
        ExistingNode n;
        for (int l = 0; l < en.n_labels; l++) {
            int k = D.key(normalize_label(en.label_keys[l]));
            n.reqs.add(D, new_req(D, k, OP_IN, {en.label_values[l]}, false, 0));
        }
        n.reqs.add(D, new_req(D, s.hostname_key, OP_IN, {en.name ? en.name : ""}, false, 0));
        for (int l = 0; l < en.n_taints; l++)
            n.taints.push_back({en.taints[l].key ? en.taints[l].key : "", en.taints[l].value ? en.taints[l].value : "",
                                en.taints[l].effect ? en.taints[l].effect : ""});
        n.available.assign(en.available, en.available + R);
        n.requests.assign(R, 0);
        if (en.requests) n.requests.assign(en.requests, en.requests + R);
        s.own_existing.push_back(std::move(n));
    }
    return KP_OK;
}

extern "C" kp_status orc_solve(const kp_catalog_view* cat, const kp_solve_input* in, kp_solve_output* out,
                               orc_result** res_out) {
    if (!cat || !in || !out) return KP_E_INVALID;
    if (in->min_values_policy != KP_MIN_VALUES_STRICT) return KP_E_UNSUPPORTED;
    auto res = std::make_unique<orc_result>();
    Solver s(res->D);
    kp_status st = parse_into(s, cat, in);
    if (st != KP_OK) return st;
    for (int j = 0; j < (int)s.own_existing.size(); j++) s.ex_idx.push_back(j);
    const kp_pods_view& pv = in->pods;
    s.plist.resize(pv.n_pods);
    for (int p = 0; p < pv.n_pods; p++) s.plist[p] = p;

    s.solve();
    s.finalize(in->max_instance_types);

    // outputs
    int n_nc = (int)s.ncs.size();
    int n_ids = 0;
    for (auto& nc : s.ncs) n_ids += (int)nc.truncated.size();
    out->n_nodeclaims = n_nc;
    out->n_type_ids = n_ids;
    out->stats = s.stats;
    if (n_nc > out->cap_nodeclaims || n_ids > out->cap_type_ids) return KP_E_BUFFER;
    std::vector<int> slice_pos(n_nc, -1);
    for (size_t i = 0; i < s.newNodeClaims.size(); i++) slice_pos[s.newNodeClaims[i]] = (int)i;
    int off = 0;
    for (int i = 0; i < n_nc; i++) {
        const NodeClaim& nc = s.ncs[i];
        out->nodeclaim_nodepool[i] = nc.valid ? s.tmpls[nc.tmpl].np_index : -1;
        out->nodeclaim_n_pods[i] = (int)nc.pods.size();
        if (out->nodeclaim_slice_pos) out->nodeclaim_slice_pos[i] = slice_pos[i];
        if (out->nodeclaim_n_options) out->nodeclaim_n_options[i] = (int)nc.options.size();
        out->nodeclaim_type_offset[i] = off;
        for (int t : nc.truncated) out->type_ids[off++] = t;
    }
    out->nodeclaim_type_offset[n_nc] = off;
    for (int p = 0; p < pv.n_pods; p++) {
        out->pod_result[p] = s.pod_result[p];
        if (out->pod_order) out->pod_order[p] = s.pod_order[p];
    }
    if (res_out) {
        res->ncs = std::move(s.ncs);
        *res_out = res.release();
    }
    return KP_OK;
}

// ------------------------------------------------------------------------------------------------
// Consolidation ([core] pkg/controllers/disruption, recalled — DESIGN.md §7)
// ------------------------------------------------------------------------------------------------
namespace orc {

struct ConsCtx {
    Solver* base;
    const kp_consolidate_input* in;
    int ct_key = -1;
    Reqs ct_reserved, ct_spot, ct_od;  // NewRequirements(capacity-type In [x])
    Req spot_req;
    int v_spot = -1, v_od = -1;        // value ids in the capacity-type dictionary
};

// Offerings.Available().WorstLaunchPrice(reqs) (cloudprovider/types.go): the first capacity type in the precedence
// reserved, spot, on-demand with a compatible offering; the most expensive such offering.
static double worst_launch_price(const ConsCtx& X, int t, const Reqs& reqs) {
    const Solver& b = *X.base;
    for (const Reqs* ct : {&X.ct_reserved, &X.ct_spot, &X.ct_od}) {
        bool any = false;
        double mx = 0;
        for (auto& o : b.ty(t).offerings) {
            if (!o.available || !reqs_compatible(b.D, reqs, o.reqs, true) || !reqs_compatible(b.D, *ct, o.reqs, true))
                continue;
            if (!any || o.price > mx) mx = o.price;
            any = true;
        }
        if (any) return mx;
    }
    return DBL_MAX;
}

// requirement.Has(value) for a value that may be absent from the dictionary
static bool req_has_vid(const Dict& D, const Reqs& reqs, int key, int vid) {
    if (key < 0) return true;
    auto it = reqs.m.find(key);
    if (it == reqs.m.end()) return true;  // undefined key: Get() is Exists
    const Req& r = it->second;
    if (vid < 0) return r.complement && !r.has_gt && !r.has_lt;
    return req_has(D, r, vid);
}

static int consolidate_probe_count(const kp_consolidate_input* in) {
    const int n = in->n_candidates;
    if (in->mode == KP_CONSOLIDATE_SINGLE) return n;
    if (n < 2) return 0;
    const int mx = in->max_candidates > 0 ? in->max_candidates : 100;
    return n <= mx ? n - 1 : mx;  // firstNConsolidationOption: mid in [1, max], prefix candidates[0 : mid+1]
}

// One SimulateScheduling + computeConsolidation (+ the multi-node filterOutSameInstanceType test).
static void run_probe(const ConsCtx& X, int probe, kp_probe_result& pr) {
    const kp_consolidate_input* in = X.in;
    const Solver& b = *X.base;
    const int c0 = in->mode == KP_CONSOLIDATE_SINGLE ? probe : 0;
    const int c1 = in->mode == KP_CONSOLIDATE_SINGLE ? probe + 1 : probe + 2;
    pr = kp_probe_result{};
    Solver s(b.D);
    s.R = b.R;
    s.cpu_axis = b.cpu_axis;
    s.mem_axis = b.mem_axis;
    s.hostname_key = b.hostname_key;
    s.host_req = b.host_req;
    s.tp = &b.own_types;
    s.cp = &b.own_classes;
    s.pp = &b.own_pods;
    s.ex_base = &b.own_existing;
    s.tmpls = b.tmpls;
    // SimulateScheduling: state nodes minus the candidates; NewScheduler recomputes NodePool remaining resources over
    // those nodes, i.e. the candidates' capacity returns to their NodePools.
    std::vector<uint8_t> excluded(b.own_existing.size(), 0);
    double cprice = 0;
    bool all_spot = true;
    for (int c = c0; c < c1; c++) {
        const kp_candidate& cd = in->candidates[c];
        excluded[cd.node] = 1;
        cprice += cd.price;  // getCandidatePrices
        if (cd.capacity_type != KP_CT_SPOT) all_spot = false;
        if (cd.capacity && cd.nodepool >= 0)
            for (auto& tm : s.tmpls)
                if (tm.np_index == cd.nodepool)
                    for (int r = 0; r < s.R; r++)
                        if (tm.limit_set[r]) tm.remaining[r] += cd.capacity[r];
    }
    for (int j = 0; j < (int)b.own_existing.size(); j++)
        if (!excluded[j]) s.ex_idx.push_back(j);
    // pods = pending + candidates' reschedulable pods
    for (int i = 0; i < in->n_pending; i++) s.plist.push_back(in->pending[i]);
    const int n_pending = (int)s.plist.size();
    for (int c = c0; c < c1; c++)
        for (int i = 0; i < in->candidates[c].n_pods; i++) s.plist.push_back(in->candidates[c].pods[i]);
    pr.n_pods = (int)s.plist.size();
    pr.candidate_price = cprice;

    s.solve();
    s.finalize(in->cluster.max_instance_types);  // Solve(...).TruncateInstanceTypes(MaxInstanceTypes)

    // Results.AllNonPendingPodsScheduled: pending pods may stay pending; a pod placed on an uninitialized existing
    // node is an error (SimulateScheduling)
    bool all = true;
    for (int li = n_pending; li < (int)s.plist.size(); li++) {
        const int r = s.pod_result[li];
        if (r == KP_POD_UNSCHEDULABLE) all = false;
        if (r <= -2 && in->initialized && !in->initialized[-2 - r]) all = false;
    }
    std::vector<int> valid;
    for (int i = 0; i < (int)s.ncs.size(); i++)
        if (s.ncs[i].valid) valid.push_back(i);
    pr.all_scheduled = all ? 1 : 0;
    pr.n_new_nodeclaims = valid.size() < 2 ? (int)valid.size() : 2;
    if (!all) return;
    if (valid.empty()) {
        pr.decision = KP_DECISION_DELETE;
        pr.valid = 1;
        return;
    }
    if (valid.size() != 1) return;  // "we're not going to turn a single node into multiple candidates"
    NodeClaim& nc = s.ncs[valid[0]];
    Reqs reqs = nc.reqs;
    std::vector<int> opts = nc.truncated;  // already OrderByPrice(reqs)
    const int ncand = c1 - c0;
    auto price_filter = [&](const Reqs& rq, double maxp) {  // RemoveInstanceTypeOptionsByPriceAndMinValues / filterByPrice
        std::vector<int> o;
        for (int t : opts)
            if (worst_launch_price(X, t, rq) < maxp) o.push_back(t);
        return o;
    };
    const bool has_spot = req_has_vid(b.D, reqs, X.ct_key, X.v_spot);
    if (all_spot && has_spot) {
        // computeSpotToSpotConsolidation
        if (!in->spot_to_spot) return;
        if (X.ct_key >= 0) reqs.add(b.D, X.spot_req);
        opts = price_filter(reqs, cprice);
        int need = 0;
        if (!s.satisfies_min_values(opts, reqs, &need)) return;
        if (opts.empty()) return;
        if (ncand == 1) {
            if ((int)opts.size() < 15) return;  // MinInstanceTypesForSpotToSpotConsolidation
            const int keep = reqs.has_min_values() ? std::max(15, need) : 15;
            if ((int)opts.size() > keep) opts.resize(keep);
        }
    } else {
        opts = price_filter(reqs, cprice);
        if (!s.satisfies_min_values(opts, reqs)) return;
        if (opts.empty()) return;
        if (has_spot && req_has_vid(b.D, reqs, X.ct_key, X.v_od) && X.ct_key >= 0) reqs.add(b.D, X.spot_req);
    }
    pr.decision = KP_DECISION_REPLACE;
    if (in->mode == KP_CONSOLIDATE_MULTI) {
        // filterOutSameInstanceType: the replacement must be cheaper than the cheapest candidate of a type it offers
        double maxp = DBL_MAX;
        for (int t : opts)
            for (int c = c0; c < c1; c++) {
                const kp_candidate& cd = in->candidates[c];
                if (cd.instance_type == t && cd.price < maxp) maxp = cd.price;
            }
        opts = price_filter(reqs, maxp);
    }
    pr.valid = opts.empty() ? 0 : 1;
    pr.n_replacement_types = (int)opts.size();
    double best = 0;
    for (size_t i = 0; i < opts.size(); i++) {
        const double w = worst_launch_price(X, opts[i], reqs);
        if (i == 0 || w < best) best = w;
    }
    pr.replacement_price = best;
}

}  // namespace orc

extern "C" int32_t orc_consolidate_probe_count(const kp_consolidate_input* in) {
    return in ? consolidate_probe_count(in) : 0;
}

extern "C" kp_status orc_consolidate(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                     kp_probe_result* results, int32_t cap_results, int32_t n_threads) {
    if (!cat || !in) return KP_E_INVALID;
    if (in->cluster.min_values_policy != KP_MIN_VALUES_STRICT) return KP_E_UNSUPPORTED;
    if (in->mode != KP_CONSOLIDATE_SINGLE && in->mode != KP_CONSOLIDATE_MULTI) return KP_E_INVALID;
    Dict D;
    Solver base(D);
    kp_status st = parse_into(base, cat, &in->cluster);
    if (st != KP_OK) return st;
    const int E = (int)base.own_existing.size(), P = (int)base.own_pods.size();
    for (int i = 0; i < in->n_pending; i++)
        if (in->pending[i] < 0 || in->pending[i] >= P) return KP_E_INVALID;
    for (int c = 0; c < in->n_candidates; c++) {
        const kp_candidate& cd = in->candidates[c];
        if (cd.node < 0 || cd.node >= E || cd.n_pods < 0 || (cd.n_pods && !cd.pods) || !(cd.price >= 0)) return KP_E_INVALID;
        for (int i = 0; i < cd.n_pods; i++)
            if (cd.pods[i] < 0 || cd.pods[i] >= P) return KP_E_INVALID;
    }
    const int np = consolidate_probe_count(in);
    const int b0 = in->probe_begin > 0 ? in->probe_begin : 0;
    const int b1 = in->probe_end > 0 && in->probe_end < np ? in->probe_end : np;
    if (b1 - b0 > cap_results) return KP_E_BUFFER;
    ConsCtx X;
    X.base = &base;
    X.in = in;
    X.ct_key = D.key("karpenter.sh/capacity-type");
    X.ct_reserved.add(D, new_req(D, X.ct_key, OP_IN, {"reserved"}, false, 0));
    X.ct_spot.add(D, new_req(D, X.ct_key, OP_IN, {"spot"}, false, 0));
    X.ct_od.add(D, new_req(D, X.ct_key, OP_IN, {"on-demand"}, false, 0));
    X.spot_req = new_req(D, X.ct_key, OP_IN, {"spot"}, false, 0);
    X.v_spot = D.value(X.ct_key, "spot");
    X.v_od = D.value(X.ct_key, "on-demand");
    // the dictionary is frozen from here on: probes only read it
    const int nt = n_threads > 1 ? n_threads : 1;
    std::atomic<int> next{b0};
    auto worker = [&]() {
        for (;;) {
            const int i = next.fetch_add(1);
            if (i >= b1) break;
            run_probe(X, i, results[i - b0]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
    return KP_OK;
}

extern "C" kp_status orc_result_nodeclaim_requirements(const orc_result* res, int32_t nc, char* buf, int64_t cap,
                                                       int64_t* needed) {
    if (!res || nc < 0 || nc >= (int)res->ncs.size()) return KP_E_INVALID;
    std::string s;
    const Dict& D = res->D;
    // canonical serialization: "key\tcomplement\tgt\tlt\tmin\tv1\x1fv2..." values sorted as strings, keys sorted
    std::vector<std::string> lines;
    for (auto& kv : res->ncs[nc].reqs.m) {
        const Req& r = kv.second;
        std::string l = D.keys[kv.first] + "\t" + (r.complement ? "1" : "0") + "\t" +
                        (r.has_gt ? std::to_string(r.gt) : "-") + "\t" + (r.has_lt ? std::to_string(r.lt) : "-") +
                        "\t" + (r.has_min ? std::to_string(r.min_values) : "-") + "\t";
        std::vector<std::string> vs;
        for (int v : r.values) vs.push_back(D.vals[kv.first][v]);
        std::sort(vs.begin(), vs.end());
        for (size_t i = 0; i < vs.size(); i++) {
            if (i) l += '\x1f';
            l += vs[i];
        }
        lines.push_back(l);
    }
    std::sort(lines.begin(), lines.end());
    for (auto& l : lines) s += l + "\n";
    if (needed) *needed = (int64_t)s.size() + 1;
    if ((int64_t)s.size() + 1 > cap) return KP_E_BUFFER;
    memcpy(buf, s.c_str(), s.size() + 1);
    return KP_OK;
}

extern "C" void orc_result_free(orc_result* res) { delete res; }
