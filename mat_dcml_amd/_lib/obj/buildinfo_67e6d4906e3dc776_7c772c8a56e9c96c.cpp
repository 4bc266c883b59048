extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "67e6d4906e3dc776";
extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "7c772c8a56e9c96c";
