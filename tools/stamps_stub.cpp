// error sink for the standalone instrumented PV library (tools/Makefile)
#include <cstdio>
extern "C" void gz_internal_set_error(const char* msg) { std::fprintf(stderr, "gz error: %s\n", msg); }
