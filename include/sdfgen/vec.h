// sdfgen/vec.h -- minimal fixed-size vector used at the C++ drop-in boundary.
// Layout-compatible with the reference's Vec<N,T> (common/vec.h:25-28: a plain
// `T v[N]`), so std::vector<Vec3f>::data() is a float[N][3] and
// std::vector<Vec3ui>::data() a uint32[N][3].  Only what callers of
// make_level_set3 need is provided.
#pragma once
#include <cstdint>

template <unsigned int N, class T>
struct Vec {
    T v[N];
    Vec() {}
    explicit Vec(T s) { for (unsigned int i = 0; i < N; ++i) v[i] = s; }
    Vec(T a, T b, T c) { static_assert(N == 3, "3-vector ctor"); v[0] = a; v[1] = b; v[2] = c; }
    T &operator[](int i) { return v[i]; }
    const T &operator[](int i) const { return v[i]; }
};

typedef Vec<3, float> Vec3f;
typedef Vec<3, unsigned int> Vec3ui;
typedef Vec<3, int> Vec3i;
static_assert(sizeof(Vec3f) == 12 && sizeof(Vec3ui) == 12, "packed 12-byte Vec3");
