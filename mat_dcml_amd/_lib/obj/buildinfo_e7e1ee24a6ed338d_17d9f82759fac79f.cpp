extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "e7e1ee24a6ed338d";
extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "17d9f82759fac79f";
