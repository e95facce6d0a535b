// kp_gosort_host.h — Go's sort.Slice on the host (Go 1.24 src/sort/slice.go + zsortfunc.go pdqsort_func).
//
// newPodRequirements ([core] scheduling/requirements.go) orders a pod's preferred node-affinity terms with
// sort.Slice(preferred, weight desc) in place and takes the first; sort.Slice is unstable beyond 12 elements
// (insertionSort_func below that), so which of several equally weighted terms comes first is part of the result.
// GoSlice<Less, Swap> reproduces pdqsort_func operation for operation over index-based less / swap callbacks.
// (The device keeps its own wave-level emulation for the in-flight NodeClaim slice: kp_gosort.h.)
#pragma once
#include <cstdint>

template <class Less, class Swap>
struct GoSlice {
    Less less;
    Swap swap;

    static int bits_len(uint64_t x) {
        int n = 0;
        for (; x; x >>= 1) n++;
        return n;
    }
    void insertion(int a, int b) {
        for (int i = a + 1; i < b; i++)
            for (int j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
    }
    void sift_down(int lo, int hi, int first) {
        for (int root = lo;;) {
            int child = 2 * root + 1;
            if (child >= hi) return;
            if (child + 1 < hi && less(first + child, first + child + 1)) child++;
            if (!less(first + root, first + child)) return;
            swap(first + root, first + child);
            root = child;
        }
    }
    void heap(int a, int b) {
        const int first = a, hi = b - a;
        for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(i, hi, first);
        for (int i = hi - 1; i >= 0; i--) {
            swap(first, first + i);
            sift_down(0, i, first);
        }
    }
    // partition_func: returns the pivot's final index; *already = no element moved
    int partition(int a, int b, int pivot, bool* already) {
        swap(a, pivot);
        int i = a + 1, j = b - 1;
        while (i <= j && less(i, a)) i++;
        while (i <= j && !less(j, a)) j--;
        if (i > j) {
            swap(j, a);
            *already = true;
            return j;
        }
        swap(i, j);
        i++;
        j--;
        for (;;) {
            while (i <= j && less(i, a)) i++;
            while (i <= j && !less(j, a)) j--;
            if (i > j) break;
            swap(i, j);
            i++;
            j--;
        }
        swap(j, a);
        *already = false;
        return j;
    }
    int partition_equal(int a, int b, int pivot) {
        swap(a, pivot);
        int i = a + 1, j = b - 1;
        for (;;) {
            while (i <= j && !less(a, i)) i++;
            while (i <= j && less(a, j)) j--;
            if (i > j) break;
            swap(i, j);
            i++;
            j--;
        }
        return i;
    }
    bool partial_insertion(int a, int b) {
        int i = a + 1;
        for (int step = 0; step < 5; step++) {
            while (i < b && !less(i, i - 1)) i++;
            if (i == b) return true;
            if (b - a < 50) return false;
            swap(i, i - 1);
            if (i - a >= 2)  // shift the smaller one left (Go's loop runs down to index 1, not a)
                for (int k = i - 1; k >= 1 && less(k, k - 1); k--) swap(k, k - 1);
            if (b - i >= 2)  // shift the greater one right
                for (int k = i + 1; k < b && less(k, k - 1); k++) swap(k, k - 1);
        }
        return false;
    }
    void break_patterns(int a, int b) {
        const int n = b - a;
        if (n < 8) return;
        uint64_t r = (uint64_t)n;  // xorshift seeded with the length
        const uint64_t mod = (uint64_t)1 << bits_len((uint64_t)n);
        const int idx = a + (n / 4) * 2 - 1;
        for (int q = 0; q < 3; q++) {
            r ^= r << 13;
            r ^= r >> 7;
            r ^= r << 17;
            int other = (int)(r & (mod - 1));
            if (other >= n) other -= n;
            swap(idx - 1 + q, a + other);
        }
    }
    // order2 / median / medianAdjacent / choosePivot: hint 0 unknown, 1 increasing, 2 decreasing
    void order2(int& x, int& y, int& swaps) {
        if (less(y, x)) {
            swaps++;
            const int t = x;
            x = y;
            y = t;
        }
    }
    int median(int a, int b, int c, int& swaps) {
        order2(a, b, swaps);
        order2(b, c, swaps);
        order2(a, b, swaps);
        return b;
    }
    void choose_pivot(int a, int b, int* pivot, int* hint) {
        const int l = b - a;
        int swaps = 0;
        int i = a + l / 4, j = a + l / 4 * 2, k = a + l / 4 * 3;
        if (l >= 8) {
            if (l >= 50) {
                i = median(i - 1, i, i + 1, swaps);
                j = median(j - 1, j, j + 1, swaps);
                k = median(k - 1, k, k + 1, swaps);
            }
            j = median(i, j, k, swaps);
        }
        *pivot = j;
        *hint = swaps == 0 ? 1 : swaps == 12 ? 2 : 0;
    }
    void pdq(int a, int b, int limit) {
        bool balanced = true, partitioned = true;
        for (;;) {
            const int n = b - a;
            if (n <= 12) {
                insertion(a, b);
                return;
            }
            if (limit == 0) {
                heap(a, b);
                return;
            }
            if (!balanced) {
                break_patterns(a, b);
                limit--;
            }
            int pivot, hint;
            choose_pivot(a, b, &pivot, &hint);
            if (hint == 2) {
                for (int i = a, j = b - 1; i < j; i++, j--) swap(i, j);
                pivot = (b - 1) - (pivot - a);
                hint = 1;
            }
            if (balanced && partitioned && hint == 1 && partial_insertion(a, b)) return;
            if (a > 0 && !less(a - 1, pivot)) {
                a = partition_equal(a, b, pivot);
                continue;
            }
            bool already = false;
            const int mid = partition(a, b, pivot, &already);
            partitioned = already;
            const int ln = mid - a, rn = b - mid;
            if (ln < rn) {
                balanced = ln >= n / 8;
                pdq(a, mid, limit);
                a = mid + 1;
            } else {
                balanced = rn >= n / 8;
                pdq(mid + 1, b, limit);
                b = mid;
            }
        }
    }
    void sort(int n) { pdq(0, n, bits_len((uint64_t)n)); }
};

template <class Less, class Swap>
inline void go_sort_slice(int n, Less less, Swap swap) {
    GoSlice<Less, Swap> s{less, swap};
    s.sort(n);
}
