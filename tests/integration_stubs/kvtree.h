/* TEST-ONLY: the one KVTree name redset's headers use (an opaque type), for
 * the adapter's syntax check (tests/test_integration_adapter.py). KVTree
 * itself is an absent third-party dependency; nothing links against this. */
#ifndef KVTREE_H
#define KVTREE_H
typedef struct kvtree_struct kvtree;
#define KVTREE_SUCCESS (0)
#endif
