// sdfgen/array3.h -- the 3-D grid of the C++ drop-in boundary.
//
// ABI contract with the reference (/root/reference/common/array3.h:24-44, 329-334): the
// class template `Array3<T, ArrayT = std::vector<T>>` in the global namespace with data
// members, in order,
//   int ni, nj, nk;   // grid dimensions
//   ArrayT a;         // flat storage, i fastest: a[i + ni*(j + nj*k)] (array3.h:114)
// and the reference's typedefs `Array3f = Array3<float, Array1<float>>` etc.  So
// `sdfgen::make_level_set3(..., Array3f &phi, ...)` mangles and lays out exactly as the
// reference's declaration (common/sdfgen_unified.h:47-57) and a caller compiled against
// either header links to libsdfgen_hip.so unchanged (tests/test_cxx_dropin.py).
#pragma once
#include <cstddef>
#include <vector>

#include "array1.h"

template <class T, class ArrayT = std::vector<T> >
struct Array3 {
    typedef typename ArrayT::iterator iterator;
    typedef typename ArrayT::const_iterator const_iterator;
    typedef typename ArrayT::size_type size_type;
    typedef long difference_type;
    typedef T &reference;
    typedef const T &const_reference;
    typedef T value_type;
    typedef T *pointer;
    typedef const T *const_pointer;

    int ni, nj, nk;
    ArrayT a;

    Array3() : ni(0), nj(0), nk(0) {}
    Array3(int ni_, int nj_, int nk_) : ni(ni_), nj(nj_), nk(nk_), a(cells(ni_, nj_, nk_)) {}
    Array3(int ni_, int nj_, int nk_, const T &value) : ni(ni_), nj(nj_), nk(nk_), a(cells(ni_, nj_, nk_), value) {}

    static size_type cells(int ni_, int nj_, int nk_) { return (size_type)ni_ * (size_type)nj_ * (size_type)nk_; }
    size_type index(int i, int j, int k) const { return (size_type)i + (size_type)ni * ((size_type)j + (size_type)nj * k); }

    T &operator()(int i, int j, int k) { return a[index(i, j, k)]; }
    const T &operator()(int i, int j, int k) const { return a[index(i, j, k)]; }
    T &operator[](size_type n) { return a[n]; }
    const T &operator[](size_type n) const { return a[n]; }

    iterator begin() { return a.begin(); }
    const_iterator begin() const { return a.begin(); }
    iterator end() { return a.end(); }
    const_iterator end() const { return a.end(); }
    size_type size() const { return a.size(); }
    bool empty() const { return a.empty(); }

    void resize(int ni_, int nj_, int nk_)
    {
        a.resize(cells(ni_, nj_, nk_));
        ni = ni_;
        nj = nj_;
        nk = nk_;
    }
    void resize(int ni_, int nj_, int nk_, const T &value)
    {
        a.resize(cells(ni_, nj_, nk_), value);
        ni = ni_;
        nj = nj_;
        nk = nk_;
    }
    void assign(const T &value)
    {
        for (size_type n = 0; n < a.size(); ++n) a[n] = value;
    }
    void assign(int ni_, int nj_, int nk_, const T &value)
    {
        resize(ni_, nj_, nk_);
        assign(value);
    }
    void clear()
    {
        a.clear();
        ni = nj = nk = 0;
    }
    void set_zero()
    {
        for (size_type n = 0; n < a.size(); ++n) a[n] = T(0);
    }
    void swap(Array3 &o)
    {
        std::swap(ni, o.ni);
        std::swap(nj, o.nj);
        std::swap(nk, o.nk);
        a.swap(o.a);
    }
};

typedef Array3<double, Array1<double> > Array3d;
typedef Array3<float, Array1<float> > Array3f;
typedef Array3<int, Array1<int> > Array3i;
typedef Array3<unsigned int, Array1<unsigned int> > Array3ui;
typedef Array3<char, Array1<char> > Array3c;
typedef Array3<unsigned char, Array1<unsigned char> > Array3uc;
