"""Diagnostic: run one small problem on the device and the oracle, print both (used while developing kernels)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import parity
from kpsim import catalog as cat, model, native, synth
fx = cat.load_fixtures()
fc = cat.fake_catalog(fx=fx)
case = fx["kats"]["gpu_packing"]["cases"][0]
pods = synth.pods_from_specs([(0, {case["resource"]: str(q)}) for q in case["requests"]])
prob = model.Problem(fc, [synth.default_nodepool()], [model.PodClass()], pods)
ctx = native.Context(0)
r, q = parity.run_device(ctx, prob)
print("DEVICE", r.n_nodeclaims, r.pod_result, r.pod_order, r.stats)
ro, qo = parity.run_oracle(prob)
print("ORACLE", ro.n_nodeclaims, ro.pod_result, ro.pod_order)
