// TEST INFRASTRUCTURE — a C++ caller of the C-ABI (include/kpsim.h), built against the CPU stub of the HIP runtime
// (hip_stub.cpp) with -fsanitize=thread by tests/cpu_stub/Makefile and run by tests/test_cpu_stub.py.
//
// It mirrors the reference's concurrency contract: instancetype.DefaultProvider.List is called from many goroutines at
// once (pkg/providers/instancetype/suite_test.go:2857-2891), and core's provisioner and disruption controllers can
// Solve concurrently.  kpsim.h promises one ctx per concurrent caller; this program checks that promise under TSAN:
//   1. N threads, one ctx each: catalog upload, kp_solve (prepare / execute / fetch), ICE / price patches,
//      kp_consolidate, kp_launch_select, all concurrently; every thread's outputs equal thread 0's;
//   2. a multi-device ctx (kp_device_opts.devices = {0, 1, 0}) used from its own thread while the others run: the
//      probe shards are gathered in global probe order (the stub reports n_pods = the probe's global index);
//   3. call-order errors: execute before prepare / consolidate_execute after a solve prepare are KP_E_STATE.
// Exit status 0 = all checks passed (TSAN's own reports make the process exit 66).
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kpsim.h"

#define CHECK(cond)                                                                                          \
    do {                                                                                                     \
        if (!(cond)) {                                                                                       \
            fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, kp_last_error(ctx)); \
            return 1;                                                                                        \
        }                                                                                                    \
    } while (0)

namespace {

// A 6-type catalog: instance-type / arch / capacity-type / zone labels, offerings over 2 zones x {on-demand, spot}.
struct Catalog {
    std::vector<const char*> res{"cpu", "memory", "pods"};
    std::vector<std::string> names;
    std::vector<const char*> name_p;
    std::vector<int64_t> cap, alloc;
    std::vector<const char*> keys{"node.kubernetes.io/instance-type", "kubernetes.io/arch", "karpenter.sh/capacity-type",
                                  "topology.kubernetes.io/zone"};
    std::vector<int8_t> state;
    std::vector<int32_t> off;
    std::vector<const char*> vals;
    std::vector<int32_t> otype, orcap;
    std::vector<double> oprice;
    std::vector<uint8_t> oavail;
    std::vector<const char*> okeys{"karpenter.sh/capacity-type", "topology.kubernetes.io/zone",
                                   "karpenter.k8s.aws/capacity-reservation-id", "karpenter.k8s.aws/capacity-reservation-type"};
    std::vector<int8_t> ostate;
    std::vector<const char*> ovals;
    kp_catalog_view v{};
    Catalog() {
        const int T = 6;
        for (int t = 0; t < T; t++) names.push_back("m9." + std::to_string(1 << t) + "xlarge");
        for (auto& n : names) name_p.push_back(n.c_str());
        for (int t = 0; t < T; t++) {
            const int64_t c = 1000LL << t, m = (int64_t)(4LL << 30) * 1000 << t;
            cap.insert(cap.end(), {c, m, 110000});
            alloc.insert(alloc.end(), {c - 80, m - (int64_t)893 * (1 << 20) * 1000, 110000});
        }
        off.push_back(0);
        for (int t = 0; t < T; t++) {
            for (int k = 0; k < 4; k++) state.push_back(KP_LABEL_IN);
            vals.push_back(name_p[t]);
            off.push_back((int32_t)vals.size());
            vals.push_back(t % 2 ? "arm64" : "amd64");
            off.push_back((int32_t)vals.size());
            vals.push_back("on-demand");
            vals.push_back("spot");
            off.push_back((int32_t)vals.size());
            vals.push_back("zone-a");
            vals.push_back("zone-b");
            off.push_back((int32_t)vals.size());
            for (int z = 0; z < 2; z++)
                for (int ct = 0; ct < 2; ct++) {
                    otype.push_back(t);
                    oprice.push_back((ct ? 0.03 : 0.1) * (1 << t) + 0.001 * z);
                    oavail.push_back(1);
                    orcap.push_back(0);
                    ostate.insert(ostate.end(), {KP_LABEL_IN, KP_LABEL_IN, KP_LABEL_DOES_NOT_EXIST, KP_LABEL_DOES_NOT_EXIST});
                    ovals.insert(ovals.end(), {ct ? "spot" : "on-demand", z ? "zone-b" : "zone-a", "", ""});
                }
        }
        v.n_types = T;
        v.n_resources = (int32_t)res.size();
        v.resource_names = res.data();
        v.type_names = name_p.data();
        v.capacity = cap.data();
        v.allocatable = alloc.data();
        v.n_label_keys = (int32_t)keys.size();
        v.label_keys = keys.data();
        v.label_state = state.data();
        v.label_offsets = off.data();
        v.label_values = vals.data();
        v.n_offerings = (int32_t)otype.size();
        v.offering_type = otype.data();
        v.offering_price = oprice.data();
        v.offering_available = oavail.data();
        v.offering_reservation_capacity = orcap.data();
        v.n_offering_keys = (int32_t)okeys.size();
        v.offering_keys = okeys.data();
        v.offering_label_state = ostate.data();
        v.offering_label_values = ovals.data();
    }
};

// 200 pods of 2 classes, one NodePool, 12 existing nodes (the consolidation cluster), 10 candidates.
struct Problem {
    const char* od_sp[2] = {"on-demand", "spot"};
    kp_requirement np_req{"karpenter.sh/capacity-type", KP_OP_IN, 2, od_sp, -1};
    kp_nodepool np{};
    const char* amd[1] = {"amd64"};
    kp_requirement cls_req{"kubernetes.io/arch", KP_OP_IN, 1, amd, -1};
    kp_pod_class cls[2]{};
    std::vector<int32_t> pod_cls;
    std::vector<int64_t> req, ts;
    std::vector<std::string> uid;
    std::vector<const char*> uid_p;
    std::vector<std::string> en_name;
    std::vector<int64_t> en_avail;
    std::vector<kp_existing_node> ex;
    std::vector<std::vector<int32_t>> cand_pods;
    std::vector<kp_candidate> cand;
    kp_solve_input in{};
    kp_consolidate_input cin{};
    Problem() {
        np.name = "default";
        np.weight = 10;
        np.n_requirements = 1;
        np.requirements = &np_req;
        np.n_types = -1;
        cls[1].n_requirements = 1;
        cls[1].requirements = &cls_req;
        const int P = 200, E = 12;
        for (int p = 0; p < P; p++) {
            pod_cls.push_back(p % 2);
            req.insert(req.end(), {(int64_t)(250 << (p % 3)), (int64_t)(512LL << 20) * 1000 * (1 + p % 4), 1000});
            ts.push_back(p);
            char b[32];
            snprintf(b, sizeof b, "pod-%05d", p);
            uid.push_back(b);
        }
        for (auto& u : uid) uid_p.push_back(u.c_str());
        for (int j = 0; j < E; j++) {
            en_name.push_back("node-" + std::to_string(j));
            en_avail.insert(en_avail.end(), {4000, (int64_t)(16LL << 30) * 1000, 110000});
        }
        for (int j = 0; j < E; j++) {
            kp_existing_node n{};
            n.name = en_name[j].c_str();
            n.available = &en_avail[(size_t)j * 3];
            ex.push_back(n);
        }
        in.n_nodepools = 1;
        in.nodepools = &np;
        in.n_classes = 2;
        in.classes = cls;
        in.pods.n_pods = P;
        in.pods.class_id = pod_cls.data();
        in.pods.requests = req.data();
        in.pods.creation_ns = ts.data();
        in.pods.uids = uid_p.data();
        in.max_instance_types = 60;
        in.min_values_policy = KP_MIN_VALUES_STRICT;
        // consolidation: the same pods bound 10 per node to the first 10 nodes, which are the candidates
        cand_pods.resize(10);
        for (int p = 0; p < 100; p++) cand_pods[p / 10].push_back(p);
        for (int c = 0; c < 10; c++) {
            kp_candidate k{};
            k.node = c;
            k.n_pods = (int32_t)cand_pods[c].size();
            k.pods = cand_pods[c].data();
            k.price = 0.1 * (c + 1);
            k.capacity_type = KP_CT_ON_DEMAND;
            k.instance_type = c % 6;
            k.nodepool = 0;
            cand.push_back(k);
        }
        cin.cluster = in;
        cin.cluster.n_existing = E;
        cin.cluster.existing = ex.data();
        cin.n_candidates = (int32_t)cand.size();
        cin.candidates = cand.data();
        cin.mode = KP_CONSOLIDATE_SINGLE;
        cin.max_candidates = 100;
    }
};

struct SolveOut {
    std::vector<int32_t> nodepool, npods, pos, nopts, toff, tids, pres, pord;
    kp_solve_output o{};
    explicit SolveOut(int P, int cap = 256) : nodepool(cap), npods(cap), pos(cap), nopts(cap), toff(cap + 1),
                                              tids(cap * 60), pres(P), pord(P) {
        o.cap_nodeclaims = cap;
        o.cap_type_ids = cap * 60;
        o.nodeclaim_nodepool = nodepool.data();
        o.nodeclaim_n_pods = npods.data();
        o.nodeclaim_slice_pos = pos.data();
        o.nodeclaim_n_options = nopts.data();
        o.nodeclaim_type_offset = toff.data();
        o.type_ids = tids.data();
        o.pod_result = pres.data();
        o.pod_order = pord.data();
    }
    bool same(const SolveOut& b) const { return o.n_nodeclaims == b.o.n_nodeclaims && pres == b.pres && pord == b.pord; }
};

int worker(const Catalog& cat, const Problem& pb, int id, int iters, std::vector<int32_t>* sig) {
    kp_ctx* ctx = nullptr;
    kp_device_opts opts{};
    opts.device = id % 2;
    CHECK(kp_ctx_create(&opts, &ctx) == KP_OK);
    CHECK(kp_catalog_upload(ctx, &cat.v, 1) == KP_OK);
    for (int it = 0; it < iters; it++) {
        SolveOut so(pb.in.pods.n_pods);
        CHECK(kp_solve(ctx, &pb.in, &so.o) == KP_OK);
        std::vector<uint8_t> av(cat.v.n_offerings, 1);
        av[(it + id) % av.size()] = 0;  // an ICE mark, then a price refresh
        CHECK(kp_catalog_patch_avail(ctx, av.data(), (int32_t)av.size(), 2 + it) == KP_OK);
        const int32_t idx[1] = {3};
        const double price[1] = {0.5 + it};
        CHECK(kp_catalog_patch_price(ctx, idx, price, 1, 2 + it) == KP_OK);
        std::vector<kp_probe_result> pr(10);
        CHECK(kp_consolidate(ctx, &pb.cin, pr.data(), 10) == KP_OK);
        for (int i = 0; i < 10; i++) CHECK(pr[i].n_pods == i);
        const char* vals[2] = {"m9.1xlarge", "m9.4xlarge"};
        kp_requirement rq{"node.kubernetes.io/instance-type", KP_OP_IN, 2, vals, -1};
        const int64_t rr[3] = {500, 0, 1000};
        kp_launch_request lr{1, &rq, rr};
        kp_launch_result res[1];
        int32_t tids[60], ovr[256];
        const kp_status ls = kp_launch_select(ctx, 1, &lr, 60, res, tids, 60, ovr, 256);
        CHECK(ls == KP_OK);
        if (it == 0) {  // a batch large enough to be pipelined over sub-batches on the ctx's worker pool
            std::vector<kp_launch_request> big(4500, lr);
            std::vector<kp_launch_result> bres(big.size());
            CHECK(kp_launch_select(ctx, (int32_t)big.size(), big.data(), 60, bres.data(), tids, 60, ovr, 256) == KP_OK);
            double st[7];
            CHECK(kp_launch_stats(ctx, st, 7) == KP_OK && st[6] == 2);
            for (const auto& r : bres) CHECK(r.n_types == 0 && r.type_offset == 0);
        }
        if (it == 0) *sig = so.pres;
        else CHECK(*sig == so.pres);
    }
    // instanceToNodeClaim write-back: offering row 1 of type 0 is (zone-a, spot)
    char lab[4096];
    int64_t need = 0, capv[3], allocv[3];
    CHECK(kp_nodeclaim_labels(ctx, 0, 1, nullptr, "default", 0, lab, sizeof lab, &need, capv, allocv) == KP_OK);
    const std::string ls(lab);
    CHECK(ls.find("karpenter.sh/capacity-type\tspot\n") != std::string::npos);
    CHECK(ls.find("topology.kubernetes.io/zone\tzone-a\n") != std::string::npos);
    CHECK(ls.find("node.kubernetes.io/instance-type\tm9.1xlarge\n") != std::string::npos);
    CHECK(ls.find("karpenter.sh/nodepool\tdefault\n") != std::string::npos);
    CHECK(capv[0] == 1000 && allocv[0] == 920);
    CHECK(kp_nodeclaim_labels(ctx, 1, 1, nullptr, nullptr, 0, lab, sizeof lab, &need, nullptr, nullptr) == KP_E_INVALID);
    CHECK(kp_ctx_destroy(ctx) == KP_OK);
    return 0;
}

int multi_device(const Catalog& cat, const Problem& pb) {
    kp_ctx* ctx = nullptr;
    const int32_t devs[3] = {0, 1, 0};
    kp_device_opts opts{};
    opts.n_devices = 3;
    opts.devices = devs;
    CHECK(kp_ctx_create(&opts, &ctx) == KP_OK);
    CHECK(kp_catalog_upload(ctx, &cat.v, 1) == KP_OK);
    for (int mode = 0; mode < 2; mode++) {
        kp_consolidate_input ci = pb.cin;
        ci.mode = mode;
        const int n = kp_consolidate_probe_count(&ci);
        CHECK(n == (mode == KP_CONSOLIDATE_SINGLE ? 10 : 9));
        std::vector<kp_probe_result> pr(n);
        CHECK(kp_consolidate(ctx, &ci, pr.data(), n) == KP_OK);
        for (int i = 0; i < n; i++) CHECK(pr[i].n_pods == i && pr[i].decision == i % 3);
        double ms[3];
        int64_t cs[16];
        CHECK(kp_consolidate_stats(ctx, ms, cs, 16) == KP_OK);
        CHECK(cs[4] == n);  // probes summed over the three shards
        // a sub-range: shards of [2, n-1) land at results[0..)
        CHECK(kp_consolidate_execute(ctx, mode, 2, n - 1, pr.data(), n) == KP_OK);
        for (int i = 0; i < n - 3; i++) CHECK(pr[i].n_pods == i + 2);
        CHECK(kp_consolidate_execute(ctx, mode, 0, 0, pr.data(), 1) == KP_E_BUFFER);
    }
    // a Solve prepare on the primary invalidates the prepared pass on every device
    CHECK(kp_solve_prepare(ctx, &pb.in) == KP_OK);
    kp_probe_result one[10];
    CHECK(kp_consolidate_execute(ctx, KP_CONSOLIDATE_SINGLE, 0, 0, one, 10) == KP_E_STATE);
    CHECK(kp_ctx_destroy(ctx) == KP_OK);
    // an ordinal past the device count fails cleanly
    const int32_t bad[2] = {0, 7};
    opts.devices = bad;
    opts.n_devices = 2;
    CHECK(kp_ctx_create(&opts, &ctx) == KP_E_DEVICE);
    return 0;
}

int call_order(const Catalog& cat, const Problem& pb) {
    kp_ctx* ctx = nullptr;
    CHECK(kp_ctx_create(nullptr, &ctx) == KP_OK);
    CHECK(kp_solve_execute(ctx) == KP_E_STATE);
    SolveOut so(pb.in.pods.n_pods);
    CHECK(kp_solve(ctx, &pb.in, &so.o) == KP_E_STATE);  // no catalog yet
    CHECK(kp_catalog_upload(ctx, &cat.v, 1) == KP_OK);
    CHECK(kp_solve_prepare(ctx, &pb.in) == KP_OK);
    kp_catalog_view broken = cat.v;
    broken.n_types = -1;
    CHECK(kp_catalog_upload(ctx, &broken, 2) != KP_OK);
    CHECK(kp_solve_execute(ctx) == KP_E_STATE);  // a failed upload drops the prepared solve
    CHECK(kp_ctx_destroy(ctx) == KP_OK);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? atoi(argv[1]) : 8, iters = argc > 2 ? atoi(argv[2]) : 4;
    Catalog cat;
    Problem pb;
    if (call_order(cat, pb)) return 1;
    kp_ctx* ctx = nullptr;  // for CHECK's message
    (void)ctx;
    std::vector<int> rc(nthreads + 1, 0);
    std::vector<std::vector<int32_t>> sig(nthreads);
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; i++) th.emplace_back([&, i] { rc[i] = worker(cat, pb, i, iters, &sig[i]); });
    th.emplace_back([&] { rc[nthreads] = multi_device(cat, pb); });
    for (auto& t : th) t.join();
    for (int i = 0; i <= nthreads; i++)
        if (rc[i]) {
            fprintf(stderr, "thread %d failed\n", i);
            return 1;
        }
    for (int i = 1; i < nthreads; i++)
        if (sig[i] != sig[0]) {
            fprintf(stderr, "thread %d result differs from thread 0\n", i);
            return 1;
        }
    printf("ok: %d threads x %d iterations + a 3-device ctx\n", nthreads, iters);
    return 0;
}
