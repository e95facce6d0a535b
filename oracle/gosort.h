// ORACLE — test infrastructure only (see oracle/README.md). Never linked into libkpsim.
//
// Restatement of Go's sort.Slice (Go 1.24, go.mod:3 of the reference): src/sort/slice.go
//   Slice(x, less) { length := rv.Len(); limit := bits.Len(uint(length)); pdqsort_func(..., 0, length, limit) }
// and the pattern-defeating quicksort in src/sort/zsortfunc.go (insertionSort_func, heapSort_func,
// pdqsort_func, partition_func, partitionEqual_func, partialInsertionSort_func, breakPatterns_func,
// choosePivot_func, median_func, medianAdjacent_func, reverseRange_func) and xorshift in sort.go.
//
// Why it matters: [core] scheduler.go re-sorts s.newNodeClaims with
//   sort.Slice(s.newNodeClaims, func(a, b int) bool { return len(..[a].Pods) < len(..[b].Pods) })
// before every in-flight placement attempt.  sort.Slice is unstable, so the exact permutation of
// equal-count NodeClaims decides first-fit.  This file reproduces it operation for operation.
#pragma once
#include <cstdint>

namespace orc {

inline int go_bits_len(uint64_t x) {
    int n = 0;
    while (x) { ++n; x >>= 1; }
    return n;
}

template <class D>
struct GoPdq {
    D& d;  // d.less(i,j), d.swap(i,j)
    explicit GoPdq(D& data) : d(data) {}

    enum Hint { unknownHint = 0, increasingHint = 1, decreasingHint = 2 };

    void insertionSort(int a, int b) {
        for (int i = a + 1; i < b; i++)
            for (int j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
    }
    void siftDown(int lo, int hi, int first) {
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
    void heapSort(int a, int b) {
        int first = a, lo = 0, hi = b - a;
        for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(i, hi, first);
        for (int i = hi - 1; i >= 0; i--) {
            d.swap(first, first + i);
            siftDown(lo, i, first);
        }
    }
    int partition(int a, int b, int pivot, bool& alreadyPartitioned) {
        d.swap(a, pivot);
        int i = a + 1, j = b - 1;
        while (i <= j && d.less(i, a)) i++;
        while (i <= j && !d.less(j, a)) j--;
        if (i > j) {
            d.swap(j, a);
            alreadyPartitioned = true;
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
        alreadyPartitioned = false;
        return j;
    }
    int partitionEqual(int a, int b, int pivot) {
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
    bool partialInsertionSort(int a, int b) {
        const int maxSteps = 5, shortestShifting = 50;
        int i = a + 1;
        for (int j = 0; j < maxSteps; j++) {
            while (i < b && !d.less(i, i - 1)) i++;
            if (i == b) return true;
            if (b - a < shortestShifting) return false;
            d.swap(i, i - 1);
            if (i - a >= 2) {
                for (int k = i - 1; k >= 1; k--) {  // NB: Go bounds this loop by 1, not a
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
    void breakPatterns(int a, int b) {
        int length = b - a;
        if (length >= 8) {
            uint64_t random = (uint64_t)length;  // xorshift(length)
            uint64_t modulus = (uint64_t)1 << go_bits_len((uint64_t)length);  // nextPowerOfTwo
            int idx = a + (length / 4) * 2 - 1;
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
    // order2_func: returns (x, y) with data[x] <= data[y]; written through x/y which may alias a/b.
    void order2(int a, int b, int& swaps, int& x, int& y) {
        const int ra = a, rb = b;
        if (d.less(rb, ra)) {
            swaps++;
            x = rb;
            y = ra;
            return;
        }
        x = ra;
        y = rb;
    }
    int median(int a, int b, int c, int& swaps) {
        order2(a, b, swaps, a, b);
        order2(b, c, swaps, b, c);
        order2(a, b, swaps, a, b);
        return b;
    }
    int medianAdjacent(int a, int& swaps) { return median(a - 1, a, a + 1, swaps); }
    void choosePivot(int a, int b, int& pivot, int& hint) {
        const int shortestNinther = 50, maxSwaps = 4 * 3;
        int l = b - a;
        int swaps = 0;
        int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
        if (l >= 8) {
            if (l >= shortestNinther) {
                i = medianAdjacent(i, swaps);
                j = medianAdjacent(j, swaps);
                k = medianAdjacent(k, swaps);
            }
            j = median(i, j, k, swaps);
        }
        pivot = j;
        if (swaps == 0) hint = increasingHint;
        else if (swaps == maxSwaps) hint = decreasingHint;
        else hint = unknownHint;
    }
    void reverseRange(int a, int b) {
        int i = a, j = b - 1;
        while (i < j) {
            d.swap(i, j);
            i++;
            j--;
        }
    }
    void pdqsort(int a, int b, int limit) {
        const int maxInsertion = 12;
        bool wasBalanced = true, wasPartitioned = true;
        for (;;) {
            int length = b - a;
            if (length <= maxInsertion) {
                insertionSort(a, b);
                return;
            }
            if (limit == 0) {
                heapSort(a, b);
                return;
            }
            if (!wasBalanced) {
                breakPatterns(a, b);
                limit--;
            }
            int pivot, hint;
            choosePivot(a, b, pivot, hint);
            if (hint == decreasingHint) {
                reverseRange(a, b);
                pivot = (b - 1) - (pivot - a);
                hint = increasingHint;
            }
            if (wasBalanced && wasPartitioned && hint == increasingHint) {
                if (partialInsertionSort(a, b)) return;
            }
            if (a > 0 && !d.less(a - 1, pivot)) {
                int mid = partitionEqual(a, b, pivot);
                a = mid;
                continue;
            }
            bool alreadyPartitioned = false;
            int mid = partition(a, b, pivot, alreadyPartitioned);
            wasPartitioned = alreadyPartitioned;
            int leftLen = mid - a, rightLen = b - mid;
            int balanceThreshold = length / 8;
            if (leftLen < rightLen) {
                wasBalanced = leftLen >= balanceThreshold;
                pdqsort(a, mid, limit);
                a = mid + 1;
            } else {
                wasBalanced = rightLen >= balanceThreshold;
                pdqsort(mid + 1, b, limit);
                b = mid;
            }
        }
    }
};

// sort.Slice(x, less) for a data adaptor d with d.size().
template <class D>
inline void go_sort_slice(D& d) {
    int n = d.size();
    GoPdq<D> s(d);
    s.pdqsort(0, n, go_bits_len((uint64_t)n));
}

}  // namespace orc
