// sdfgen/vec.h -- fixed-size vector of the C++ drop-in boundary.
//
// ABI contract with the reference (/root/reference/common/vec.h:25-28): the
// type is the class template `Vec<unsigned int N, class T>` in the global
// namespace holding exactly `T v[N]`, so
//   * `sdfgen::make_level_set3(const std::vector<Vec3ui>&, const std::vector<Vec3f>&,
//      const Vec3f&, ...)` mangles to the same linker symbol whichever of the two
//     headers a caller compiled against, and
//   * std::vector<Vec3f>::data() is a packed float[n][3] (std::vector<Vec3ui>: uint32[n][3]),
//     which is how the library reads the mesh without a copy.
// The arithmetic callers use around make_level_set3 (bounding boxes and grid sizing in
// app/main.cpp:104-251, tests/test_utils.cpp:276-305) is provided with the reference's
// evaluation order (component-wise, sums left to right; vec.h:92-157, 216-255, 331-337,
// 377-383, 545-556), so sizing computed with this header gives the reference's bits.
#pragma once
#include <cmath>
#include <cstdint>
#include <iostream>

template <unsigned int N, class T>
struct Vec {
    T v[N];

    Vec() {}
    explicit Vec(T s) { for (unsigned int i = 0; i < N; ++i) v[i] = s; }
    template <class S>
    explicit Vec(const S *src) { for (unsigned int i = 0; i < N; ++i) v[i] = (T)src[i]; }
    template <class S>
    explicit Vec(const Vec<N, S> &o) { for (unsigned int i = 0; i < N; ++i) v[i] = (T)o[i]; }
    Vec(T a, T b) { static_assert(N == 2, "Vec: two-component constructor"); v[0] = a; v[1] = b; }
    Vec(T a, T b, T c) { static_assert(N == 3, "Vec: three-component constructor"); v[0] = a; v[1] = b; v[2] = c; }
    Vec(T a, T b, T c, T d)
    {
        static_assert(N == 4, "Vec: four-component constructor");
        v[0] = a; v[1] = b; v[2] = c; v[3] = d;
    }

    T &operator[](int i) { return v[i]; }
    const T &operator[](int i) const { return v[i]; }

    bool nonzero() const
    {
        for (unsigned int i = 0; i < N; ++i)
            if (v[i]) return true;
        return false;
    }

    // Compound and binary arithmetic, one component at a time (no reassociation).
    Vec &operator+=(const Vec &w) { for (unsigned int i = 0; i < N; ++i) v[i] += w.v[i]; return *this; }
    Vec &operator-=(const Vec &w) { for (unsigned int i = 0; i < N; ++i) v[i] -= w.v[i]; return *this; }
    Vec &operator*=(const Vec &w) { for (unsigned int i = 0; i < N; ++i) v[i] *= w.v[i]; return *this; }
    Vec &operator/=(const Vec &w) { for (unsigned int i = 0; i < N; ++i) v[i] /= w.v[i]; return *this; }
    Vec &operator*=(T s) { for (unsigned int i = 0; i < N; ++i) v[i] *= s; return *this; }
    Vec &operator/=(T s) { for (unsigned int i = 0; i < N; ++i) v[i] /= s; return *this; }

    Vec operator+(const Vec &w) const { Vec r(*this); return r += w; }
    Vec operator-(const Vec &w) const { Vec r(*this); return r -= w; }
    Vec operator*(const Vec &w) const { Vec r(*this); return r *= w; }
    Vec operator/(const Vec &w) const { Vec r(*this); return r /= w; }
    Vec operator*(T s) const { Vec r(*this); return r *= s; }
    Vec operator/(T s) const { Vec r(*this); return r /= s; }
    Vec operator-() const
    {
        Vec r;
        for (unsigned int i = 0; i < N; ++i) r.v[i] = -v[i];
        return r;
    }
};

typedef Vec<2, float> Vec2f;
typedef Vec<2, double> Vec2d;
typedef Vec<2, int> Vec2i;
typedef Vec<3, float> Vec3f;
typedef Vec<3, double> Vec3d;
typedef Vec<3, int> Vec3i;
typedef Vec<3, unsigned int> Vec3ui;
typedef Vec<4, float> Vec4f;
static_assert(sizeof(Vec3f) == 12 && sizeof(Vec3ui) == 12, "Vec3 must be a packed 12-byte POD");

template <unsigned int N, class T>
inline Vec<N, T> operator*(T s, const Vec<N, T> &a) { return a * s; }

template <unsigned int N, class T>
inline bool operator==(const Vec<N, T> &a, const Vec<N, T> &b)
{
    for (unsigned int i = 0; i < N; ++i)
        if (!(a[i] == b[i])) return false;
    return true;
}
template <unsigned int N, class T>
inline bool operator!=(const Vec<N, T> &a, const Vec<N, T> &b) { return !(a == b); }

// Left-to-right sums: ((a0*b0 + a1*b1) + a2*b2) ...
template <unsigned int N, class T>
inline T dot(const Vec<N, T> &a, const Vec<N, T> &b)
{
    T s = a[0] * b[0];
    for (unsigned int i = 1; i < N; ++i) s += a[i] * b[i];
    return s;
}
template <unsigned int N, class T>
inline T mag2(const Vec<N, T> &a) { return dot(a, a); }
template <unsigned int N, class T>
inline T mag(const Vec<N, T> &a) { return std::sqrt(mag2(a)); }
template <unsigned int N, class T>
inline T dist2(const Vec<N, T> &a, const Vec<N, T> &b)
{
    T d = a[0] - b[0], s = d * d;
    for (unsigned int i = 1; i < N; ++i) { d = a[i] - b[i]; s += d * d; }
    return s;
}
template <unsigned int N, class T>
inline T dist(const Vec<N, T> &a, const Vec<N, T> &b) { return std::sqrt(dist2(a, b)); }

template <class T>
inline Vec<3, T> cross(const Vec<3, T> &a, const Vec<3, T> &b)
{
    return Vec<3, T>(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}

// Smallest / largest component.
template <unsigned int N, class T>
inline T min(const Vec<N, T> &a)
{
    T m = a[0];
    for (unsigned int i = 1; i < N; ++i) if (a[i] < m) m = a[i];
    return m;
}
template <unsigned int N, class T>
inline T max(const Vec<N, T> &a)
{
    T m = a[0];
    for (unsigned int i = 1; i < N; ++i) if (a[i] > m) m = a[i];
    return m;
}

// Grow the box [lo, hi] to contain x (component-wise; a NaN component is ignored, as
// with the reference's compare-and-assign form).
template <unsigned int N, class T>
inline void update_minmax(const Vec<N, T> &x, Vec<N, T> &lo, Vec<N, T> &hi)
{
    for (unsigned int i = 0; i < N; ++i) {
        if (x[i] < lo[i]) lo[i] = x[i];
        else if (x[i] > hi[i]) hi[i] = x[i];
    }
}
template <unsigned int N, class T>
inline void minmax(const Vec<N, T> &a, const Vec<N, T> &b, Vec<N, T> &lo, Vec<N, T> &hi)
{
    for (unsigned int i = 0; i < N; ++i) {
        if (a[i] < b[i]) { lo[i] = a[i]; hi[i] = b[i]; }
        else { lo[i] = b[i]; hi[i] = a[i]; }
    }
}
template <unsigned int N, class T>
inline void minmax(const Vec<N, T> &a, const Vec<N, T> &b, const Vec<N, T> &c, Vec<N, T> &lo, Vec<N, T> &hi)
{
    minmax(a, b, lo, hi);
    update_minmax(c, lo, hi);
}

template <unsigned int N, class T>
inline std::ostream &operator<<(std::ostream &out, const Vec<N, T> &a)
{
    out << a[0];
    for (unsigned int i = 1; i < N; ++i) out << ' ' << a[i];
    return out;
}
template <unsigned int N, class T>
inline std::istream &operator>>(std::istream &in, Vec<N, T> &a)
{
    for (unsigned int i = 0; i < N; ++i) in >> a[i];
    return in;
}
