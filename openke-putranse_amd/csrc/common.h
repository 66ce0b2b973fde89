// Shared host-side plumbing of libputranse_hip.so: status codes, last-error text, HIP checks.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "putranse.h"

namespace pt {

void set_error(int code, const std::string &msg);
int fail(int code, const std::string &msg);   // records and returns code

#define PT_HIP(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return ::pt::fail(PT_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

#define PT_CHECK(cond, code, msg)                 \
    do {                                          \
        if (!(cond)) return ::pt::fail(code, msg); \
    } while (0)

}  // namespace pt
