"""kpsim — host side of the MI355X-native Karpenter scheduling-simulation library.

The compute path is libkpsim.so (HIP kernels for gfx950 behind the C-ABI in include/kpsim.h); this
package marshals the reference's scheduling inputs (cloudprovider.InstanceType catalog, NodePools, pods)
into that ABI and mirrors the reference's Solve() entry point.
"""
