for v in b256 b512 b1024 b256 b512 b1024; do FBN_LIB_PATH=tools/variants/lib_$v.so timeout -k 10 120 python tools/time_fields.py 2>/dev/null | grep fields_fwd || exit 1; done
