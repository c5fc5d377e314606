/*
 * Redundancy-file header trees for the offline rebuild tool: the C side of
 * redset_amd/header.py (same text form, same RSHIPHDR frame).
 *
 * A tree is redset's kvtree shape: every node has a key and children; a
 * "KEY = VALUE" pair is a node KEY with one childless child VALUE. Text form
 * = kvtree_print's layout (doc/rst/schemes.rst:262-327, :520-603), children
 * in strcmp order as redset_sort_kvtree leaves them (src/redset_util.c:191).
 */
#ifndef REDSET_HIP_HEADER_TREE_H
#define REDSET_HIP_HEADER_TREE_H

#include <stddef.h>

typedef struct htree {
  char* key;
  struct htree** kids;
  int n, cap;
} htree;

htree* ht_new(const char* key);
void ht_free(htree* t);
htree* ht_copy(const htree* t);
/* child by key, NULL if absent */
htree* ht_get(const htree* t, const char* key);
/* child by key, created if absent */
htree* ht_child(htree* t, const char* key);
/* attach an existing subtree (takes ownership; replaces a same-key child) */
void ht_put(htree* t, htree* sub);
/* the single value of KEY (its only child's key), NULL if absent/ambiguous */
const char* ht_val(const htree* t, const char* key);
/* value of KEY as an integer; returns -1 when absent or malformed */
int ht_ull(const htree* t, const char* key, unsigned long long* out);
/* set KEY = VALUE (replacing) */
void ht_set_ull(htree* t, const char* key, unsigned long long v);

/* text form (malloc'd, NUL-terminated) and its parser */
char* ht_render(const htree* t);
htree* ht_parse(const char* text);

/* framed header I/O: "RSHIPHDR", u64 LE body length, text + NUL.
 * read: returns the tree and sets *header_size; NULL on a bad/short header.
 * write: writes at the fd's position, returns bytes written or -1. */
htree* ht_read_header(int fd, unsigned long long* header_size);
long long ht_write_header(int fd, const htree* t);

#endif
