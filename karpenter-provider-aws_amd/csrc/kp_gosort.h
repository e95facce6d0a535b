// kp_gosort.h — exact emulation of Go's sort.Slice over the in-flight NodeClaim slice, in LDS.
//
// [core] scheduler.go calls sort.Slice(s.newNodeClaims, by len(Pods) asc) before every in-flight placement.
// sort.Slice is Go 1.24's pdqsort_func (src/sort/zsortfunc.go): unstable, so the permutation of NodeClaims with
// equal pod counts is part of the observable result (it decides first-fit).  Between two sorts exactly one
// element changes (one NodeClaim gains a pod, or one is appended with 1 pod), so:
//   * no inversion                → pdqsort leaves the slice untouched;
//   * n <= 12                     → insertionSort = the stable move of the changed element;
//   * n >= 50 and choosePivot's samples show no inversion (increasing hint) → partialInsertionSort, which for a
//                                   single displaced element also performs exactly the stable move;
//   * otherwise                   → the full pdqsort_func emulation (pdqsort_full), operation for operation.
// The stable move is a rotation of one run of equal keys, done by a whole wave.
#pragma once
#include "kp_device.h"

// Slice keys carry the FFD rejection memo in bit 31 (the NodeClaim rejected the current pod shape); comparisons
// use the low 31 bits = len(Pods).
#define KEYMASK 0x7FFFFFFFu

struct SortSlice {
    uint32_t* key;  // len(Pods) by slice position (| KEY_REJ)
    uint16_t* ord;  // NodeClaim id by slice position
    __device__ bool less(int i, int j) const { return (key[i] & KEYMASK) < (key[j] & KEYMASK); }
    __device__ void swap(int i, int j) {
        const uint32_t k = key[i];
        key[i] = key[j];
        key[j] = k;
        const uint16_t o = ord[i];
        ord[i] = ord[j];
        ord[j] = o;
    }
};

__device__ __forceinline__ int go_bits_len(unsigned x) { return x ? 32 - __clz(x) : 0; }

// The same slice held one element per lane (n <= 64): compares and swaps are readlanes on wave-uniform indices,
// so the pdqsort emulation runs as scalar control flow without LDS round trips.
struct RegSlice {
    uint32_t k;
    uint32_t o;
    int lane;
    __device__ __forceinline__ bool less(int i, int j) const {
        return ((uint32_t)__builtin_amdgcn_readlane((int)k, i) & KEYMASK) <
               ((uint32_t)__builtin_amdgcn_readlane((int)k, j) & KEYMASK);
    }
    __device__ __forceinline__ void swap(int i, int j) {
        const uint32_t ki = __builtin_amdgcn_readlane((int)k, i), kj = __builtin_amdgcn_readlane((int)k, j);
        const uint32_t oi = __builtin_amdgcn_readlane((int)o, i), oj = __builtin_amdgcn_readlane((int)o, j);
        if (lane == i) {
            k = kj;
            o = oj;
        } else if (lane == j) {
            k = ki;
            o = oi;
        }
    }
};

// order2_func / median_func / medianAdjacent_func / choosePivot_func (one lane)
template <class D>
__device__ inline void go_order2(const D& d, int a, int b, int& swaps, int& x, int& y) {
    if (d.less(b, a)) {
        swaps++;
        x = b;
        y = a;
    } else {
        x = a;
        y = b;
    }
}
template <class D>
__device__ inline int go_median(const D& d, int a, int b, int c, int& swaps) {
    int x, y;
    go_order2(d, a, b, swaps, x, y);
    a = x;
    b = y;
    go_order2(d, b, c, swaps, x, y);
    b = x;
    c = y;
    go_order2(d, a, b, swaps, x, y);
    return y;
}
// hint: 0 unknown, 1 increasing, 2 decreasing
template <class D>
__device__ inline void go_choose_pivot(const D& d, int a, int b, int& pivot, int& hint) {
    const int l = b - a;
    int swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
        if (l >= 50) {
            i = go_median(d, i - 1, i, i + 1, swaps);
            j = go_median(d, j - 1, j, j + 1, swaps);
            k = go_median(d, k - 1, k, k + 1, swaps);
        }
        j = go_median(d, i, j, k, swaps);
    }
    pivot = j;
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
}

// Same swaps count as go_choose_pivot(0, n) but with the ≤ 9 sampled keys loaded by lanes in parallel.
__device__ inline int choose_pivot_hint_wave(const SortSlice& d, int n, int lane) {
    const int l = n, i = l / 4, j = l / 4 * 2, k = l / 4 * 3;
    int p = 0;
    if (l >= 50) {
        const int q = lane % 3, g = lane / 3;
        p = (g == 0 ? i : g == 1 ? j : k) - 1 + q;
    } else {
        p = lane == 0 ? i : lane == 1 ? j : k;
    }
    const int nl = l >= 50 ? 9 : 3;
    const uint32_t kv = (lane < nl) ? (d.key[p] & KEYMASK) : 0u;
    uint32_t v[9];
#pragma unroll
    for (int q = 0; q < 9; q++) v[q] = __builtin_amdgcn_readlane(kv, q);
    int swaps = 0;
    // median on (value) triples; only the order of values matters for the swap count and the chosen element
    auto med = [&](uint32_t a, uint32_t b, uint32_t c) -> uint32_t {
        uint32_t x, y;
        if (b < a) { swaps++; x = b; y = a; } else { x = a; y = b; }
        a = x; b = y;
        if (c < b) { swaps++; x = c; y = b; } else { x = b; y = c; }
        b = x; c = y;
        if (b < a) { swaps++; x = b; y = a; } else { x = a; y = b; }
        return y;
    };
    if (l >= 50) {
        const uint32_t mi = med(v[0], v[1], v[2]);
        const uint32_t mj = med(v[3], v[4], v[5]);
        const uint32_t mk = med(v[6], v[7], v[8]);
        med(mi, mj, mk);
    } else if (l >= 8) {
        med(v[0], v[1], v[2]);
    }
    return swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
}

template <class D>
__device__ inline void go_insertion_sort(D& d, int a, int b) {
    for (int i = a + 1; i < b; i++)
        for (int j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
}
template <class D>
__device__ inline void go_sift_down(D& d, int lo, int hi, int first) {
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
template <class D>
__device__ inline void go_heap_sort(D& d, int a, int b) {
    const int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) go_sift_down(d, i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
        d.swap(first, first + i);
        go_sift_down(d, lo, i, first);
    }
}
template <class D>
__device__ inline int go_partition(D& d, int a, int b, int pivot, bool& already) {
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
template <class D>
__device__ inline int go_partition_equal(D& d, int a, int b, int pivot) {
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
template <class D>
__device__ inline bool go_partial_insertion_sort(D& d, int a, int b) {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
        while (i < b && !d.less(i, i - 1)) i++;
        if (i == b) return true;
        if (b - a < 50) return false;
        d.swap(i, i - 1);
        if (i - a >= 2) {
            for (int k = i - 1; k >= 1; k--) {  // Go bounds this loop by 1, not a
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
template <class D>
__device__ inline void go_break_patterns(D& d, int a, int b) {
    const int length = b - a;
    if (length >= 8) {
        uint64_t random = (uint64_t)length;  // xorshift(length)
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
template <class D>
__device__ inline void go_reverse_range(D& d, int a, int b) {
    int i = a, j = b - 1;
    while (i < j) {
        d.swap(i, j);
        i++;
        j--;
    }
}
// pdqsort_func(data, 0, n, bits.Len(n)) with Go's recursion order (smaller side first) on an explicit stack.
template <class D>
__device__ inline void pdqsort_full(D& d, int n, int* stk) {
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
        int a = __builtin_amdgcn_readfirstlane(stk[sp * 5 + 0]), b = __builtin_amdgcn_readfirstlane(stk[sp * 5 + 1]);
        int limit = __builtin_amdgcn_readfirstlane(stk[sp * 5 + 2]);
        bool wasBalanced = __builtin_amdgcn_readfirstlane(stk[sp * 5 + 3]) != 0;
        bool wasPartitioned = __builtin_amdgcn_readfirstlane(stk[sp * 5 + 4]) != 0;
        for (;;) {
            const int length = b - a;
            if (length <= 12) {
                go_insertion_sort(d, a, b);
                break;
            }
            if (limit == 0) {
                go_heap_sort(d, a, b);
                break;
            }
            if (!wasBalanced) {
                go_break_patterns(d, a, b);
                limit--;
            }
            int pivot, hint;
            go_choose_pivot(d, a, b, pivot, hint);
            if (hint == 2) {
                go_reverse_range(d, a, b);
                pivot = (b - 1) - (pivot - a);
                hint = 1;
            }
            if (wasBalanced && wasPartitioned && hint == 1) {
                if (go_partial_insertion_sort(d, a, b)) break;
            }
            if (a > 0 && !d.less(a - 1, pivot)) {
                a = go_partition_equal(d, a, b, pivot);
                continue;
            }
            bool already = false;
            const int mid = go_partition(d, a, b, pivot, already);
            wasPartitioned = already;
            const int leftLen = mid - a, rightLen = b - mid;
            const int balanceThreshold = length / 8;
            if (leftLen < rightLen) {
                wasBalanced = leftLen >= balanceThreshold;
                push(mid + 1, b, limit, wasBalanced, wasPartitioned);  // the loop continues here afterwards
                push(a, mid, limit, 1, 1);                             // recursive pdqsort_func first
            } else {
                wasBalanced = rightLen >= balanceThreshold;
                push(a, mid, limit, wasBalanced, wasPartitioned);
                push(mid + 1, b, limit, 1, 1);
            }
            break;
        }
    }
}

// ---- wave-parallel pieces of the stable move ----
__device__ inline int wave_find_first_ge(const SortSlice& d, int s, int n, uint32_t v, int lane) {
    for (int base = s; base < n; base += 64) {
        const int p = base + lane;
        const uint64_t m = __ballot(p < n && (d.key[p] & KEYMASK) >= v);
        if (m) return base + __ffsll((unsigned long long)m) - 1;
    }
    return n;
}
__device__ inline int wave_find_first_gt(const SortSlice& d, int s, int n, uint32_t v, int lane) {
    for (int base = s; base < n; base += 64) {
        const int p = base + lane;
        const uint64_t m = __ballot(p < n && (d.key[p] & KEYMASK) > v);
        if (m) return base + __ffsll((unsigned long long)m) - 1;
    }
    return n;
}
// [a, e): element a moves to e-1, the rest shift left by one
__device__ inline void wave_rotate_left(SortSlice& d, int a, int e, int lane) {
    if (e - a < 2) return;
    const uint16_t fo = d.ord[a];
    const uint32_t fk = d.key[a];
    for (int base = a; base < e - 1; base += 64) {
        const int i = base + lane;
        uint16_t o = 0;
        uint32_t k = 0;
        if (i < e - 1) {
            o = d.ord[i + 1];
            k = d.key[i + 1];
        }
        asm volatile("" ::: "memory");
        if (i < e - 1) {
            d.ord[i] = o;
            d.key[i] = k;
        }
        asm volatile("" ::: "memory");
    }
    if (lane == 0) {
        d.ord[e - 1] = fo;
        d.key[e - 1] = fk;
    }
}
// [q, n): element n-1 moves to q, the rest shift right by one
__device__ inline void wave_rotate_right(SortSlice& d, int q, int n, int lane) {
    if (n - q < 2) return;
    const uint16_t lo = d.ord[n - 1];
    const uint32_t lk = d.key[n - 1];
    for (int top = n - 1; top > q; top -= 64) {
        const int i = top - lane;
        uint16_t o = 0;
        uint32_t k = 0;
        if (i > q) {
            o = d.ord[i - 1];
            k = d.key[i - 1];
        }
        asm volatile("" ::: "memory");
        if (i > q) {
            d.ord[i] = o;
            d.key[i] = k;
        }
        asm volatile("" ::: "memory");
    }
    if (lane == 0) {
        d.ord[q] = lo;
        d.key[q] = lk;
    }
}

// The slice in LDS driven by the whole wave: control flow is wave-uniform (keys are read with readfirstlane), the
// O(n) scans of partition / partitionEqual / partialInsertionSort become 64-wide ballot searches, and swaps are
// written by lane 0.  Same comparison outcomes and swap sequence as Go, hence the same permutation.
struct WaveLds {
    uint32_t* key;
    uint16_t* ord;
    int lane;
    __device__ __forceinline__ uint32_t k(int i) const { return (uint32_t)__builtin_amdgcn_readfirstlane((int)key[i]) & KEYMASK; }
    __device__ __forceinline__ bool less(int i, int j) const { return k(i) < k(j); }
    __device__ __forceinline__ void swap(int i, int j) {
        const uint32_t ki = key[i], kj = key[j];
        const uint16_t oi = ord[i], oj = ord[j];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane == 0) {
            key[i] = kj;
            key[j] = ki;
            ord[i] = oj;
            ord[j] = oi;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    // first q in [lo, hi] with pred(masked key[q]) (hi + 1 if none)
    template <class F>
    __device__ __forceinline__ int find_first(int lo, int hi, F pred) const {
        for (int base = lo; base <= hi; base += 64) {
            const int q = base + lane;
            const uint64_t m = __ballot(q <= hi && pred(key[q] & KEYMASK));
            if (m) return base + __ffsll((unsigned long long)m) - 1;
        }
        return hi + 1;
    }
    // last q in [lo, hi] with pred(masked key[q]) (lo - 1 if none)
    template <class F>
    __device__ __forceinline__ int find_last(int lo, int hi, F pred) const {
        for (int top = hi; top >= lo; top -= 64) {
            const int q = top - lane;
            const uint64_t m = __ballot(q >= lo && pred(key[q] & KEYMASK));
            if (m) return top - (__ffsll((unsigned long long)m) - 1);
        }
        return lo - 1;
    }
    // [a, e): element a moves to e-1, the rest shift left by one
    __device__ __forceinline__ void rotl(int a, int e) {
        if (e - a < 2) return;
        const uint32_t fk = key[a];
        const uint16_t fo = ord[a];
        for (int base = a; base < e - 1; base += 64) {
            const int i = base + lane;
            uint32_t kx = 0;
            uint16_t ox = 0;
            if (i < e - 1) {
                kx = key[i + 1];
                ox = ord[i + 1];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (i < e - 1) {
                key[i] = kx;
                ord[i] = ox;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (lane == 0) {
            key[e - 1] = fk;
            ord[e - 1] = fo;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    // [q, n): element n-1 moves to q, the rest shift right by one
    __device__ __forceinline__ void rotr(int q, int n) {
        if (n - q < 2) return;
        const uint32_t lk = key[n - 1];
        const uint16_t lo = ord[n - 1];
        for (int top = n - 1; top > q; top -= 64) {
            const int i = top - lane;
            uint32_t kx = 0;
            uint16_t ox = 0;
            if (i > q) {
                kx = key[i - 1];
                ox = ord[i - 1];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (i > q) {
                key[i] = kx;
                ord[i] = ox;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (lane == 0) {
            key[q] = lk;
            ord[q] = lo;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
};

// partition_func with wave scans
__device__ inline int go_partition(WaveLds& d, int a, int b, int pivot, bool& already) {
    d.swap(a, pivot);
    const uint32_t pk = d.k(a);
    int i = a + 1, j = b - 1;
    i = d.find_first(i, j, [&](uint32_t x) { return !(x < pk); });  // while i <= j && less(data[i], data[a]) i++
    j = d.find_last(i, j, [&](uint32_t x) { return x < pk; });      // while i <= j && !less(data[j], data[a]) j--
    if (i > j) {
        d.swap(j, a);
        already = true;
        return j;
    }
    d.swap(i, j);
    i++;
    j--;
    for (;;) {
        i = d.find_first(i, j, [&](uint32_t x) { return !(x < pk); });
        j = d.find_last(i, j, [&](uint32_t x) { return x < pk; });
        if (i > j) break;
        d.swap(i, j);
        i++;
        j--;
    }
    d.swap(j, a);
    already = false;
    return j;
}
// partitionEqual_func with wave scans
__device__ inline int go_partition_equal(WaveLds& d, int a, int b, int pivot) {
    d.swap(a, pivot);
    const uint32_t pk = d.k(a);
    int i = a + 1, j = b - 1;
    for (;;) {
        i = d.find_first(i, j, [&](uint32_t x) { return pk < x; });   // while i <= j && !less(data[a], data[i]) i++
        j = d.find_last(i, j, [&](uint32_t x) { return !(pk < x); }); // while i <= j && less(data[a], data[j]) j--
        if (i > j) break;
        d.swap(i, j);
        i++;
        j--;
    }
    return i;
}
// partialInsertionSort_func with wave scans; the two shift loops are single-element moves (rotations)
__device__ inline bool go_partial_insertion_sort(WaveLds& d, int a, int b) {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
        // while i < b && !less(data[i], data[i-1]) i++
        {
            int r = b;
            for (int base = i; base < b; base += 64) {
                const int q = base + d.lane;
                const uint64_t m = __ballot(q < b && (d.key[q] & KEYMASK) < (d.key[q - 1] & KEYMASK));
                if (m) {
                    r = base + __ffsll((unsigned long long)m) - 1;
                    break;
                }
            }
            i = r;
        }
        if (i == b) return true;
        if (b - a < 50) return false;
        d.swap(i, i - 1);
        if (i - a >= 2) {
            // for k := i-1; k >= 1 && less(data[k], data[k-1]); k-- { swap(k, k-1) }: x = data[i-1] moves left past
            // the larger keys before it (Go bounds this loop by 1, not a)
            const uint32_t x = d.k(i - 1);
            const int t = d.find_last(0, i - 2, [&](uint32_t y) { return !(x < y); });  // last position not > x
            int dst = t + 1;
            d.rotr(dst, i);
        }
        if (b - i >= 2) {
            // for k := i+1; k < b && less(data[k], data[k-1]); k++ { swap(k, k-1) }: x = data[i] moves right past
            // the smaller keys after it
            const uint32_t x = d.k(i);
            const int t = d.find_first(i + 1, b - 1, [&](uint32_t y) { return !(y < x); });
            d.rotl(i, t);
        }
    }
    return false;
}
__device__ inline void go_reverse_range(WaveLds& d, int a, int b) {
    const int n = b - a, h = n / 2;
    for (int base = 0; base < h; base += 64) {
        const int i = base + d.lane;
        uint32_t ki = 0, kj = 0;
        uint16_t oi = 0, oj = 0;
        if (i < h) {
            ki = d.key[a + i];
            kj = d.key[b - 1 - i];
            oi = d.ord[a + i];
            oj = d.ord[b - 1 - i];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (i < h) {
            d.key[a + i] = kj;
            d.key[b - 1 - i] = ki;
            d.ord[a + i] = oj;
            d.ord[b - 1 - i] = oi;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

// Full pdqsort_func emulation: in registers for n <= 64, else on lane 0 over LDS.
__device__ inline void pdqsort_any(SortSlice d, int n, int* stk, int lane) {
    if (n <= 64) {
        RegSlice r;
        r.lane = lane;
        r.k = lane < n ? d.key[lane] : 0u;
        r.o = lane < n ? d.ord[lane] : 0u;
        pdqsort_full(r, n, stk);
        if (lane < n) {
            d.key[lane] = r.k;
            d.ord[lane] = (uint16_t)r.o;
        }
        return;
    }
    WaveLds w{d.key, d.ord, lane};
    pdqsort_full(w, n, stk);
}

// Is `pos` one of the positions choosePivot samples for a slice of length n >= 50 (l/4·{1,2,3} ± 1)?
__device__ __forceinline__ bool is_pivot_sample(int n, int pos) {
    const int q = n / 4;
    const int d1 = pos - q, d2 = pos - 2 * q, d3 = pos - 3 * q;
    return (d1 >= -1 && d1 <= 1) || (d2 >= -1 && d2 <= 1) || (d3 >= -1 && d3 <= 1);
}

// sort.Slice after one change (kind 1: element at pos gained a pod; kind 2: element appended at n-1).
// Returns 0 nothing to do, 1 fast stable move, 2 full emulation (done by lane 0).  One wave, all lanes.
//
// The slice was sorted before the change and only position pos moved, so choosePivot's 9 samples can show a
// swap only if pos is one of them: elsewhere the hint is "increasing" without loading them.  The stable move of
// kind 1 is one LDS round trip when the run it crosses is shorter than 64: every lane loads one (key, ord) after
// pos, the ballot gives the run end e, and lanes shift [pos+1, e) left by one.
__device__ inline int sort_slice_after_change(SortSlice d, int n, int kind, int pos, int* stk, int lane) {
    if (kind == 0 || n <= 1) return 0;
    if (kind == 1) {
        if (pos + 1 >= n) return 0;
        const uint32_t kr = d.key[pos], kv = kr & KEYMASK;
        const int q = pos + 1 + lane;
        uint32_t k = 0xFFFFFFFFu;
        uint16_t o = 0;
        if (q < n) {
            k = d.key[q];
            o = d.ord[q];
        }
        const uint64_t ge = __ballot((k & KEYMASK) >= kv || q >= n);  // lanes past n count as >=
        if (ge & 1ull) return 0;                // key[pos+1] >= key[pos]: no inversion
        bool fast = n <= 12;
        if (!fast) fast = n >= 50 && (!is_pivot_sample(n, pos) || choose_pivot_hint_wave(d, n, lane) == 1);
        if (!fast) {
            pdqsort_any(d, n, stk, lane);
            return 2;
        }
        if (ge) {
            const int first = __ffsll((unsigned long long)ge) - 1;  // run end e = pos + 1 + first
            const uint16_t mo = d.ord[pos];
            if (lane < first) {
                d.key[pos + lane] = k;
                d.ord[pos + lane] = o;
            }
            if (lane == 0) {
                d.key[pos + first] = kr;
                d.ord[pos + first] = mo;
            }
            return 1;
        }
        const int e = wave_find_first_ge(d, pos + 1, n, kv, lane);
        wave_rotate_left(d, pos, e, lane);
        return 1;
    }
    const bool inv = (d.key[n - 2] & KEYMASK) > (d.key[n - 1] & KEYMASK);
    if (!inv) return 0;
    bool fast = n <= 12;
    if (!fast) fast = n >= 50 && (!is_pivot_sample(n, n - 1) || choose_pivot_hint_wave(d, n, lane) == 1);
    if (fast) {
        const int q = wave_find_first_gt(d, 0, n - 1, d.key[n - 1] & KEYMASK, lane);
        wave_rotate_right(d, q, n, lane);
        return 1;
    }
    pdqsort_any(d, n, stk, lane);
    return 2;
}
