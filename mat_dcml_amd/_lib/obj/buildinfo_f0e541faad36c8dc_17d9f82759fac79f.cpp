extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "f0e541faad36c8dc";
extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "17d9f82759fac79f";
