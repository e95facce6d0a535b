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
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
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
    std::vector<InstanceType> types;
    std::vector<Template> tmpls;
    std::vector<PodClass> classes;
    std::vector<Pod> pods;
    std::vector<ExistingNode> existing;
    std::vector<NodeClaim> ncs;       // creation order
    std::vector<int> newNodeClaims;   // s.newNodeClaims slice (indices into ncs)
    std::vector<int> pod_result, pod_order;
    int placements = 0;
    int hostname_key = -1;
    int64_t nodeID = 0;
    kp_solve_stats stats{};

    explicit Solver(Dict& d) : D(d) {}

    // compatible(it, reqs) = it.Requirements.Intersects(reqs) == nil
    bool compatible(const InstanceType& it, const Reqs& reqs) const { return reqs_intersects(D, it.reqs, reqs); }
    bool has_offering(const InstanceType& it, const Reqs& reqs) const {
        for (auto& o : it.offerings)
            if (o.available && reqs_compatible(D, reqs, o.reqs, true)) return true;
        return false;
    }
    // InstanceTypes.SatisfiesMinValues(requirements) == nil
    bool satisfies_min_values(const std::vector<int>& its, const Reqs& reqs) const {
        for (auto& kv : reqs.m) {
            if (!kv.second.has_min) continue;
            std::vector<int> seen;
            for (int t : its) {
                Req r = types[t].reqs.get(kv.first);
                for (int v : r.values) seen.push_back(v);
            }
            std::sort(seen.begin(), seen.end());
            seen.erase(std::unique(seen.begin(), seen.end()), seen.end());
            if ((int)seen.size() < kv.second.min_values) return false;
        }
        return true;
    }
    // filterInstanceTypesByRequirements (MIN_VALUES_POLICY=Strict)
    std::vector<int> filter(const std::vector<int>& its, const Reqs& reqs, const std::vector<int64_t>& total) const {
        std::vector<int> out;
        for (int t : its) {
            const InstanceType& it = types[t];
            if (compatible(it, reqs) && fits(total, it.alloc) && has_offering(it, reqs)) out.push_back(t);
        }
        if (reqs.has_min_values() && !satisfies_min_values(out, reqs)) out.clear();
        return out;
    }

    bool nodeclaim_add(NodeClaim& nc, int p) {
        const Pod& pod = pods[p];
        const PodClass& pc = classes[pod.cls];
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
        nc.pods.push_back(p);
        nc.options.swap(remaining);
        nc.requests.swap(requests);
        nc.reqs = std::move(r);
        return true;
    }

    bool existing_add(ExistingNode& n, int p) {
        const Pod& pod = pods[p];
        const PodClass& pc = classes[pod.cls];
        if (!tolerates_all(n.taints, pc.tols)) return false;
        std::vector<int64_t> requests(R);
        for (int k = 0; k < R; k++) requests[k] = n.requests[k] + pod.req[k];
        if (!fits(requests, n.available)) return false;
        Reqs r = n.reqs;
        if (!reqs_compatible(D, r, pc.reqs, false)) return false;
        r.add_all(D, pc.reqs);
        n.requests.swap(requests);
        n.reqs = std::move(r);
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

    bool add(int p) {
        for (size_t j = 0; j < existing.size(); j++) {
            stats.existing_evals++;
            if (existing_add(existing[j], p)) {
                pod_result[p] = KP_POD_EXISTING((int)j);
                return true;
            }
        }
        SliceAdaptor sa{this};
        go_sort_slice(sa);
        stats.nodeclaim_candidates_scanned += (int64_t)newNodeClaims.size();
        for (int idx : newNodeClaims) {
            stats.nodeclaim_evals++;
            if (nodeclaim_add(ncs[idx], p)) {
                pod_result[p] = idx;
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
                    if (tm.limit_set[k] && types[t].cap[k] > tm.remaining[k]) viable = false;
                if (viable) its.push_back(t);
            }
            if (its.empty()) continue;
            // NewNodeClaim
            NodeClaim nc;
            nc.id = (int)ncs.size();
            nc.tmpl = (int)ti;
            nc.reqs = tm.reqs;
            char host[64];
            snprintf(host, sizeof host, "hostname-placeholder-%04lld", (long long)(++nodeID));
            nc.reqs.add(D, new_req(D, hostname_key, OP_IN, {host}, false, 0));
            nc.options = its;
            nc.requests = tm.daemon;
            stats.template_evals++;
            if (!nodeclaim_add(nc, p)) continue;
            // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
            for (int k = 0; k < R; k++) {
                if (!tm.limit_set[k]) continue;
                int64_t mx = 0;
                bool first = true;
                for (int t : nc.options) {
                    if (first || types[t].cap[k] > mx) mx = types[t].cap[k];
                    first = false;
                }
                tm.remaining[k] -= mx;
            }
            ncs.push_back(std::move(nc));
            newNodeClaims.push_back((int)ncs.size() - 1);
            pod_result[p] = (int)ncs.size() - 1;
            return true;
        }
        return false;
    }

    void solve() {
        // NewQueue: sort.Slice(pods, byCPUAndMemoryDescending) — a total order (UIDs unique).
        std::vector<int> order(pods.size());
        for (size_t i = 0; i < pods.size(); i++) order[i] = (int)i;
        std::sort(order.begin(), order.end(), [&](int a, int b) {
            const Pod& l = pods[a];
            const Pod& r = pods[b];
            if (l.req[cpu_axis] != r.req[cpu_axis]) return l.req[cpu_axis] > r.req[cpu_axis];
            if (l.req[mem_axis] != r.req[mem_axis]) return l.req[mem_axis] > r.req[mem_axis];
            if (l.ts != r.ts) return l.ts < r.ts;
            return l.uid < r.uid;
        });
        std::deque<int> q(order.begin(), order.end());
        std::unordered_map<int, int> lastLen;
        pod_result.assign(pods.size(), KP_POD_UNSCHEDULABLE);
        pod_order.assign(pods.size(), -1);
        for (;;) {
            if (q.empty()) break;
            int p = q.front();
            auto it = lastLen.find(p);
            if (it != lastLen.end() && it->second == (int)q.size()) break;
            q.pop_front();
            stats.pods_popped++;
            if (add(p)) {
                pod_order[p] = placements++;
                continue;
            }
            // preferences.Relax: no preferred terms in this build's inputs → never relaxed
            q.push_back(p);
            lastLen[p] = (int)q.size();
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

extern "C" kp_status orc_solve(const kp_catalog_view* cat, const kp_solve_input* in, kp_solve_output* out,
                               orc_result** res_out) {
    if (!cat || !in || !out) return KP_E_INVALID;
    if (in->min_values_policy != KP_MIN_VALUES_STRICT) return KP_E_UNSUPPORTED;
    auto res = std::make_unique<orc_result>();
    Dict& D = res->D;
    Solver s(D);
    const int T = cat->n_types, R = cat->n_resources;
    s.R = R;
    s.cpu_axis = s.mem_axis = -1;
    for (int r = 0; r < R; r++) {
        if (!strcmp(cat->resource_names[r], "cpu")) s.cpu_axis = r;
        if (!strcmp(cat->resource_names[r], "memory")) s.mem_axis = r;
    }
    if (s.cpu_axis < 0 || s.mem_axis < 0) return KP_E_INVALID;
    s.hostname_key = D.key("kubernetes.io/hostname");
    // catalog → []*cloudprovider.InstanceType
    s.types.resize(T);
    for (int t = 0; t < T; t++) {
        InstanceType& it = s.types[t];
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
        s.types[t].offerings.push_back(std::move(of));
    }
    // pod classes
    s.classes.resize(in->n_classes);
    for (int c = 0; c < in->n_classes; c++) {
        const kp_pod_class& pc = in->classes[c];
        if (!build_reqs(D, pc.requirements, pc.n_requirements, s.classes[c].reqs)) return KP_E_INVALID;
        for (int i = 0; i < pc.n_tolerations; i++) {
            Toleration t;
            t.key = pc.tolerations[i].key ? pc.tolerations[i].key : "";
            t.op = pc.tolerations[i].op;
            t.value = pc.tolerations[i].value ? pc.tolerations[i].value : "";
            t.effect = pc.tolerations[i].effect ? pc.tolerations[i].effect : "";
            s.classes[c].tols.push_back(t);
        }
    }
    // pods
    const kp_pods_view& pv = in->pods;
    s.pods.resize(pv.n_pods);
    for (int p = 0; p < pv.n_pods; p++) {
        Pod& pod = s.pods[p];
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
        s.existing.push_back(std::move(n));
    }

    s.solve();

    // FinalizeScheduling + Results.TruncateInstanceTypes(maxInstanceTypes)
    for (auto& nc : s.ncs) {
        nc.reqs.m.erase(s.hostname_key);
        // OrderByPrice(reqs)
        std::vector<std::pair<double, int>> keyed;
        for (int t : nc.options) {
            double price = DBL_MAX;
            bool any = false;
            for (auto& o : s.types[t].offerings) {
                if (!o.available || !reqs_compatible(D, nc.reqs, o.reqs, true)) continue;
                if (!any || o.price < price) price = o.price;
                any = true;
            }
            keyed.push_back({any ? price : DBL_MAX, t});
        }
        std::sort(keyed.begin(), keyed.end(), [&](const std::pair<double, int>& a, const std::pair<double, int>& b) {
            if (a.first == b.first) return s.types[a.second].name < s.types[b.second].name;
            return a.first < b.first;
        });
        std::vector<int> tr;
        for (auto& kv : keyed) tr.push_back(kv.second);
        if (in->max_instance_types > 0 && (int)tr.size() > in->max_instance_types) tr.resize(in->max_instance_types);
        if (nc.reqs.has_min_values() && !s.satisfies_min_values(tr, nc.reqs)) {
            nc.valid = false;
            for (int p : nc.pods) {
                s.pod_result[p] = KP_POD_UNSCHEDULABLE;
                s.pod_order[p] = -1;
            }
        }
        nc.truncated = tr;
    }

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
