// All model families of SURVEY.md §2.2 have native graphs (raft_stereo.cpp, crestereo.cpp,
// hitnet.cpp, fast_acvnet.cpp); presets are dispatched in runtime/engine.cpp.
