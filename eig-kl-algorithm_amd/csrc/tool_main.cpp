// main() of the cEIG / cKL / gKL / gKL2 executables: the tool name is fixed
// at build time (-DEK_TOOL="cKL"), the logic lives in libeigkl_hip.so.
#include "../../include/eigkl.h"

#ifndef EK_TOOL
#define EK_TOOL "cKL"
#endif

int main(int argc, char** argv) { return ek_cli_main(EK_TOOL, argc, argv); }
