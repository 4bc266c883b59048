extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "b64ed48c3ca4ac83";
extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "17d9f82759fac79f";
