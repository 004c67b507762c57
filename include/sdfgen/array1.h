// sdfgen/array1.h -- 1-D storage of the C++ drop-in's Array3f.
//
// ABI contract with the reference (/root/reference/common/array1.h:58-80): the class
// template `Array1<T>` in the global namespace whose only data members are, in order,
//   unsigned long n;      // element count
//   unsigned long max_n;  // capacity
//   T *data;              // C heap block (calloc/malloc/realloc; released with free)
// Same layout and the same allocator family, so an Array3f built and destroyed by a caller
// compiled against the reference's headers may be resized by this library and vice versa.
// It is a plain-old-data container: elements are not constructed or destroyed.
// Only the std::vector-like subset that callers of make_level_set3 and the .sdf writers
// touch is provided (size/resize/reserve/assign/fill/indexing/iteration/swap).
#pragma once
#include <climits>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <new>
#include <utility>

template <typename T>
struct Array1 {
    typedef T *iterator;
    typedef const T *const_iterator;
    typedef unsigned long size_type;
    typedef long difference_type;
    typedef T &reference;
    typedef const T &const_reference;
    typedef T value_type;
    typedef T *pointer;
    typedef const T *const_pointer;
    typedef std::reverse_iterator<iterator> reverse_iterator;
    typedef std::reverse_iterator<const_iterator> const_reverse_iterator;

    unsigned long n;
    unsigned long max_n;
    T *data;

    Array1() : n(0), max_n(0), data(nullptr) {}
    explicit Array1(unsigned long count) : n(0), max_n(0), data(nullptr) { alloc_zeroed(count); }
    Array1(unsigned long count, const T &value) : n(0), max_n(0), data(nullptr)
    {
        alloc_zeroed(count);
        for (unsigned long i = 0; i < n; ++i) data[i] = value;
    }
    Array1(unsigned long count, const T *src) : n(0), max_n(0), data(nullptr)
    {
        alloc_zeroed(count);
        if (count) std::memcpy(data, src, count * sizeof(T));
    }
    Array1(const Array1 &o) : n(0), max_n(0), data(nullptr)
    {
        alloc_zeroed(o.n);
        if (o.n) std::memcpy(data, o.data, o.n * sizeof(T));
    }
    ~Array1() { std::free(data); }

    Array1 &operator=(const Array1 &o)
    {
        if (this != &o) {
            if (o.n > max_n) reserve_exact(o.n);
            n = o.n;
            if (n) std::memcpy(data, o.data, n * sizeof(T));
        }
        return *this;
    }

    T &operator[](unsigned long i) { return data[i]; }
    const T &operator[](unsigned long i) const { return data[i]; }
    T &operator()(unsigned long i) { return data[i]; }
    const T &operator()(unsigned long i) const { return data[i]; }
    T &at(unsigned long i) { return data[i]; }
    const T &at(unsigned long i) const { return data[i]; }

    iterator begin() { return data; }
    const_iterator begin() const { return data; }
    iterator end() { return data + n; }
    const_iterator end() const { return data + n; }
    reverse_iterator rbegin() { return reverse_iterator(end()); }
    reverse_iterator rend() { return reverse_iterator(begin()); }
    T &front() { return data[0]; }
    T &back() { return data[n - 1]; }

    unsigned long size() const { return n; }
    unsigned long capacity() const { return max_n; }
    bool empty() const { return n == 0; }
    unsigned long max_size() const { return ULONG_MAX / sizeof(T); }

    // Capacity becomes exactly r (grow or shrink), contents kept up to min(n, r).
    void reserve(unsigned long r) { reserve_exact(r); }
    void resize(unsigned long count)
    {
        if (count > max_n) reserve_exact(count);
        n = count;
    }
    void resize(unsigned long count, const T &value)
    {
        if (count > max_n) reserve_exact(count);
        for (unsigned long i = n; i < count; ++i) data[i] = value;
        n = count;
    }
    void assign(const T &value) { for (unsigned long i = 0; i < n; ++i) data[i] = value; }
    void assign(unsigned long count, const T &value) { fill(count, value); }
    void fill(unsigned long count, const T &value)
    {
        if (count > max_n) {
            std::free(data);
            data = nullptr;
            max_n = n = 0;
            if (count > max_size()) throw std::bad_alloc();
            data = static_cast<T *>(std::malloc(count * sizeof(T)));
            if (!data && count) throw std::bad_alloc();
            max_n = count;
        }
        n = count;
        for (unsigned long i = 0; i < n; ++i) data[i] = value;
    }
    void set_zero() { if (n) std::memset(data, 0, n * sizeof(T)); }
    void clear()
    {
        std::free(data);
        data = nullptr;
        n = max_n = 0;
    }
    void push_back(const T &value)
    {
        if (n == max_n) reserve_exact(max_n * 2 + 1);
        data[n++] = value;
    }
    void pop_back() { --n; }
    void swap(Array1 &o)
    {
        std::swap(n, o.n);
        std::swap(max_n, o.max_n);
        std::swap(data, o.data);
    }

    bool operator==(const Array1 &o) const
    {
        if (n != o.n) return false;
        for (unsigned long i = 0; i < n; ++i)
            if (!(data[i] == o.data[i])) return false;
        return true;
    }
    bool operator!=(const Array1 &o) const { return !(*this == o); }

private:
    void alloc_zeroed(unsigned long count)
    {
        if (count > max_size()) throw std::bad_alloc();
        if (count == 0) return;
        data = static_cast<T *>(std::calloc(count, sizeof(T)));
        if (!data) throw std::bad_alloc();
        n = max_n = count;
    }
    void reserve_exact(unsigned long r)
    {
        if (r > max_size()) throw std::bad_alloc();
        T *p = static_cast<T *>(std::realloc(data, r * sizeof(T)));
        if (!p && r) throw std::bad_alloc();
        data = p;
        max_n = r;
        if (n > r) n = r;
    }
};

typedef Array1<double> Array1d;
typedef Array1<float> Array1f;
typedef Array1<int> Array1i;
typedef Array1<unsigned int> Array1ui;
typedef Array1<char> Array1c;
typedef Array1<unsigned char> Array1uc;
