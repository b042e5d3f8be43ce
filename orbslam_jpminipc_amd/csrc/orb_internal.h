// orb_internal.h — host-side plumbing shared by the translation units of liborb_hip.so
// (not part of the C ABI).
#pragma once
#include <string>

// Records `msg` as the calling thread's orb_last_error() and returns `code`.
__attribute__((visibility("hidden"))) int orb_internal_set_error(int code, const std::string& msg);
