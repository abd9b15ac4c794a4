// bin/exe/bfs -- drop-in for the reference's src/main/c/src/algorithms/bfs.cpp executable.
#include "common.h"

int main(int argc, char **argv) { return gxexe::Main(argc, argv, gxexe::Algorithm::BFS); }
