// bin/exe/sssp -- drop-in for the reference's src/main/c/src/algorithms/sssp.cpp executable.
#include "common.h"

int main(int argc, char **argv) { return gxexe::Main(argc, argv, gxexe::Algorithm::SSSP); }
