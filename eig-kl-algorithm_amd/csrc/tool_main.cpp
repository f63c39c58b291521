// main() of the cEIG / cKL / gKL / gKL2 executables: the tool name is fixed
// at build time (-DEK_TOOL="cKL"), the logic lives in libeigkl_hip.so.
// A short run's GPU context (~0.35 GB at ibm18 shape) is left to the process
// exit: every result is written and flushed and every stream drained when
// ek_cli_main_ex returns, and the runtime's orderly teardown (hipFree of the
// context, HSA shutdown in the static destructors) cost ~0.2 s of a 0.45 s
// fresh-process run (tools/cold_probe.py).
#include <cstdio>
#include <unistd.h>

#include "../../include/eigkl.h"

#ifndef EK_TOOL
#define EK_TOOL "cKL"
#endif

int main(int argc, char** argv) {
    const int rc = ek_cli_main_ex(EK_TOOL, argc, argv, EK_CLI_NO_TEARDOWN);
    std::fflush(nullptr);
    _exit(rc);
}
