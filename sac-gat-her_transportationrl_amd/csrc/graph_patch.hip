// graph_patch.hip -- make captured HIP graphs replay-safe on ROCm 7.2.
//
// The trainer replays its whole SAC update from a HIP graph (train.py,
// GraphedUpdate).  On this stack the CLR graph packet-capture path replays
// memset nodes smaller than ~1 MiB incorrectly from the second replay on (the
// fill does not happen), and torch's multi-block reductions clear their
// inter-block semaphores with exactly such a hipMemsetAsync -- so column
// sums (bias gradients) and similar reductions return garbage
// (tools/graph_memset_check.py reproduces it).  Kernel and memcpy nodes are
// fine, and disabling packet capture altogether makes every replay ~30x
// slower to launch.  trx_graph_patch_memsets rewrites each memset node of a
// captured (not yet instantiated) graph into an equivalent fill-kernel node
// with the same dependencies, before the graph is instantiated.
#include <hip/hip_runtime.h>

#include <vector>

#include "trx_internal.h"

namespace trx {

// hipMemsetParams semantics: `height` rows of `width` elements of
// `element_size` bytes (1, 2 or 4), rows `pitch` bytes apart, each element
// set to the low element_size bytes of `value`.
__global__ void __launch_bounds__(256) graph_fill_kernel(char* __restrict__ dst, unsigned element_size,
                                                         size_t width, size_t height, size_t pitch, unsigned value) {
    const size_t total = width * height;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t row = i / width, col = i - row * width;
        char* p = dst + row * pitch + col * element_size;
        if (element_size == 4)
            *reinterpret_cast<unsigned*>(p) = value;
        else if (element_size == 2)
            *reinterpret_cast<unsigned short*>(p) = (unsigned short)value;
        else
            *p = (char)value;
    }
}

hipError_t patch_graph_memsets(hipGraph_t graph, int* n_patched) {
    *n_patched = 0;
    size_t n = 0;
    hipError_t e = hipGraphGetNodes(graph, nullptr, &n);
    if (e != hipSuccess) return e;
    std::vector<hipGraphNode_t> nodes(n);
    if (n && (e = hipGraphGetNodes(graph, nodes.data(), &n)) != hipSuccess) return e;
    for (hipGraphNode_t node : nodes) {
        hipGraphNodeType type;
        if ((e = hipGraphNodeGetType(node, &type)) != hipSuccess) return e;
        if (type != hipGraphNodeTypeMemset) continue;
        hipMemsetParams mp;
        if ((e = hipGraphMemsetNodeGetParams(node, &mp)) != hipSuccess) return e;
        size_t nd = 0, nt = 0;
        if ((e = hipGraphNodeGetDependencies(node, nullptr, &nd)) != hipSuccess) return e;
        std::vector<hipGraphNode_t> deps(nd);
        if (nd && (e = hipGraphNodeGetDependencies(node, deps.data(), &nd)) != hipSuccess) return e;
        if ((e = hipGraphNodeGetDependentNodes(node, nullptr, &nt)) != hipSuccess) return e;
        std::vector<hipGraphNode_t> outs(nt);
        if (nt && (e = hipGraphNodeGetDependentNodes(node, outs.data(), &nt)) != hipSuccess) return e;

        char* dst = static_cast<char*>(mp.dst);
        unsigned esize = mp.elementSize;
        size_t width = mp.width, height = mp.height ? mp.height : 1, pitch = mp.pitch;
        unsigned value = mp.value;
        if (esize != 1 && esize != 2 && esize != 4) return hipErrorInvalidValue;
        if (height == 1) pitch = width * esize;
        const size_t total = width * height;
        unsigned blocks = (unsigned)((total + 255) / 256);
        if (blocks > 2048) blocks = 2048;
        if (blocks == 0) blocks = 1;
        void* args[] = {&dst, &esize, &width, &height, &pitch, &value};
        hipKernelNodeParams kp = {};
        kp.func = reinterpret_cast<void*>(graph_fill_kernel);
        kp.gridDim = dim3(blocks);
        kp.blockDim = dim3(256);
        kp.sharedMemBytes = 0;
        kp.kernelParams = args;
        kp.extra = nullptr;
        hipGraphNode_t kn;
        if ((e = hipGraphAddKernelNode(&kn, graph, nd ? deps.data() : nullptr, nd, &kp)) != hipSuccess) return e;
        for (hipGraphNode_t o : outs)
            if ((e = hipGraphAddDependencies(graph, &kn, &o, 1)) != hipSuccess) return e;
        if ((e = hipGraphDestroyNode(node)) != hipSuccess) return e;
        ++*n_patched;
    }
    return hipSuccess;
}

}  // namespace trx
