// host_io.hpp -- host-only helpers of the C ABI's file writers (dna_io.cpp),
// kept free of HIP headers so that the same units build under the host
// ASan/UBSan harness (tests/asan/).
#pragma once
#include <cstddef>
#include <string>

namespace ldpc {

// thread-local error string behind ldpc_last_error() (capi.cpp; the sanitizer
// harness defines its own)
void set_error(const std::string& msg);

// Python repr(float) of v into out (at least 32 bytes, no terminator); returns
// the length.
size_t py_float_repr(double v, char* out);

}  // namespace ldpc
