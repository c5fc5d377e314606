/* TEST-ONLY: the one KVTree name redset's headers use (an opaque type), for
 * compiling the adapter (tests/test_integration_adapter.py, tests/adapter/).
 * KVTree itself is an absent third-party dependency; nothing calls into it. */
#ifndef KVTREE_H
#define KVTREE_H
typedef struct kvtree_struct kvtree;
#define KVTREE_SUCCESS (0)
#endif
