// Tuning and diagnostic switches.
//
// The product library (lib/libsfmx.so) reads no environment variable: there
// SFMX_DIAG_ENV(name) is a null pointer and the variable's name is not even
// compiled in, so a stray variable cannot change what the library computes.
// The diagnostic build (`make diag` -> lib/libsfmx_diag.so, -DSFMX_DIAG) reads
// them: A/B timing of kernel variants, the variant parity tests
// (tests/diag.py loads that library next to the product one), and the
// alternative BA factorization forms.  Variants that are timing probes with
// wrong results exist only in that build.
#pragma once

#ifdef SFMX_DIAG
#include <cstdlib>
#define SFMX_DIAG_ENV(name) std::getenv(name)
#else
#define SFMX_DIAG_ENV(name) (static_cast<const char*>(nullptr))
#endif
