extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "67e6d4906e3dc776";
extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "cdfa317a7b3e99dc";
