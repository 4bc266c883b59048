extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "180b60274f174447";
extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "17d9f82759fac79f";
