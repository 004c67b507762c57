// sdfgen/array3.h -- minimal 3-D array used at the C++ drop-in boundary.
// Same storage contract as the reference's Array3<T> (common/array3.h:24-127):
// dims ni, nj, nk (int) and a flat std::vector<T> `a` indexed i-fastest,
// a[i + ni*(j + nj*k)].
#pragma once
#include <cstddef>
#include <vector>

template <class T>
struct Array3 {
    int ni = 0, nj = 0, nk = 0;
    std::vector<T> a;
    Array3() {}
    Array3(int ni_, int nj_, int nk_) : ni(ni_), nj(nj_), nk(nk_), a((size_t)ni_ * nj_ * nk_) {}
    Array3(int ni_, int nj_, int nk_, const T &v) : ni(ni_), nj(nj_), nk(nk_), a((size_t)ni_ * nj_ * nk_, v) {}
    T &operator()(int i, int j, int k) { return a[(size_t)i + (size_t)ni * ((size_t)j + (size_t)nj * k)]; }
    const T &operator()(int i, int j, int k) const { return a[(size_t)i + (size_t)ni * ((size_t)j + (size_t)nj * k)]; }
    void resize(int ni_, int nj_, int nk_) { ni = ni_; nj = nj_; nk = nk_; a.resize((size_t)ni_ * nj_ * nk_); }
    void assign(const T &v) { std::fill(a.begin(), a.end(), v); }
    T *data() { return a.data(); }
    const T *data() const { return a.data(); }
    size_t size() const { return a.size(); }
};

typedef Array3<float> Array3f;
typedef Array3<int> Array3i;
