// ORACLE — test infrastructure only.  Force-included (g++ -include) ahead of
// the unchanged /root/reference/cKL.cpp by oracle/ref.mk to build
// oracle/_ref/cKL_seeded.  cKL seeds its random initial split from
// std::random_device (cKL.cpp:179-180), so a random-init run can never be
// replayed; this puts a device that returns $EK_REF_SEED in its place, and
// nothing else changes (the mt19937 + std::shuffle split, cKL.cpp:180-191,
// and the rest of the program are the reference's own code).
#include <cstdlib>
#include <random>

struct ek_seeded_random_device {
    unsigned int operator()() const {
        const char* s = std::getenv("EK_REF_SEED");
        return s ? static_cast<unsigned int>(std::strtoul(s, nullptr, 10)) : 0u;
    }
};
#define random_device ek_seeded_random_device
