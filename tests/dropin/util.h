// tests/dropin/util.h — TEST INFRASTRUCTURE: a restatement (not a copy) of the caller-side
// src/util.h that stays in an unchanged reference build (util.h:1-80): IndexType is a class of one
// 32-bit word with a user-provided copy constructor, as Xilinx ap_uint<32> is (so it is passed by
// reference, not in a register, by the C++ ABI), ComputeUnits / VectFactor come from -DCU / -DVF,
// BusDataType is a 16-byte class. Only what main.cpp and csr.h use is restated.
#ifndef DROPIN_TEST_UTIL_H
#define DROPIN_TEST_UTIL_H
#include <stdint.h>
#include <sys/time.h>

struct IndexType {
    uint32_t v;
    IndexType(uint32_t x = 0) : v(x) {}
    IndexType(const IndexType &o) : v(o.v) {}  // user-provided, like ap_uint's
    IndexType &operator=(const IndexType &o) { v = o.v; return *this; }
    operator uint32_t() const { return v; }
};
#define INDEX_TYPE_BIT_WIDTH 32

#if DOUBLE == 0
typedef float ValueType;
#define VALUE_TYPE_BIT_WIDTH 32
#else
typedef double ValueType;
#define VALUE_TYPE_BIT_WIDTH 64
#endif

#define VectFactor VF
#define ComputeUnits CU
#define BUS_BIT_WIDTH 128
struct BusDataType {
    uint64_t w[2];
};

double getTimestamp();
#endif
