// integration/ie_dropin.hpp -- shared by the drop-in translation units: the
// reference's own classes with their loops replaced by calls into the MI355X library.
//
// One device context per process (an inline function's static: one instance across the drop-in
// objects), created on first use on device 0, as the reference's single-threaded main() needs.
#ifndef IE_DROPIN_HPP
#define IE_DROPIN_HPP

#include <cstdint>

#include "MatrixReader.hpp"
#include "ie_hip.h"

namespace ie_dropin {

inline ie_ctx* gpu() {
    static ie_ctx* c = [] {
        ie_ctx* p = nullptr;
        return ie_create(0, &p) == IE_OK ? p : nullptr;
    }();
    return c;
}

// MatrixReader<>::getData (MatrixReader.cpp:195-198) holds the matrix as doubles of uint16 values
inline int set_quant(ie_ctx* c, dc::MatrixReader<>& m) {
    uint16_t q[dc::BlockSize * dc::BlockSize];
    for (size_t k = 0; k < dc::BlockSize * dc::BlockSize; k++) q[k] = uint16_t(m.getData()[k]);
    return ie_set_quant(c, q, int(dc::BlockSize));
}

}  // namespace ie_dropin

#endif
