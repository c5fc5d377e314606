/* Redundancy-file header trees (see header_tree.h; mirrors redset_amd/header.py). */
#include "header_tree.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static const char MAGIC[8] = {'R', 'S', 'H', 'I', 'P', 'H', 'D', 'R'};

htree* ht_new(const char* key) {
  htree* t = calloc(1, sizeof(htree));
  t->key = strdup(key ? key : "");
  return t;
}

void ht_free(htree* t) {
  if (!t) return;
  for (int i = 0; i < t->n; ++i) ht_free(t->kids[i]);
  free(t->kids);
  free(t->key);
  free(t);
}

static void push(htree* t, htree* sub) {
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 4;
    t->kids = realloc(t->kids, (size_t) t->cap * sizeof(htree*));
  }
  t->kids[t->n++] = sub;
}

htree* ht_copy(const htree* t) {
  htree* c = ht_new(t->key);
  for (int i = 0; i < t->n; ++i) push(c, ht_copy(t->kids[i]));
  return c;
}

htree* ht_get(const htree* t, const char* key) {
  if (!t) return NULL;
  for (int i = 0; i < t->n; ++i)
    if (strcmp(t->kids[i]->key, key) == 0) return t->kids[i];
  return NULL;
}

htree* ht_child(htree* t, const char* key) {
  htree* c = ht_get(t, key);
  if (!c) {
    c = ht_new(key);
    push(t, c);
  }
  return c;
}

void ht_put(htree* t, htree* sub) {
  for (int i = 0; i < t->n; ++i)
    if (strcmp(t->kids[i]->key, sub->key) == 0) {
      ht_free(t->kids[i]);
      t->kids[i] = sub;
      return;
    }
  push(t, sub);
}

const char* ht_val(const htree* t, const char* key) {
  const htree* c = ht_get(t, key);
  return c && c->n == 1 ? c->kids[0]->key : NULL;
}

int ht_ull(const htree* t, const char* key, unsigned long long* out) {
  const char* v = ht_val(t, key);
  if (!v || !*v) return -1;
  char* end;
  unsigned long long x = strtoull(v, &end, 10);
  if (*end) return -1;
  *out = x;
  return 0;
}

void ht_set_ull(htree* t, const char* key, unsigned long long v) {
  char buf[32];
  snprintf(buf, sizeof(buf), "%llu", v);
  htree* c = ht_new(key);
  push(c, ht_new(buf));
  ht_put(t, c);
}

/* ------------------------------------------------------------ text form */

typedef struct {
  char* p;
  size_t n, cap;
} sbuf;

static void sput(sbuf* b, const char* s, size_t len) {
  if (b->n + len + 1 > b->cap) {
    while (b->n + len + 1 > b->cap) b->cap = b->cap ? 2 * b->cap : 4096;
    b->p = realloc(b->p, b->cap);
  }
  memcpy(b->p + b->n, s, len);
  b->n += len;
  b->p[b->n] = 0;
}

static int by_key(const void* a, const void* b) {
  return strcmp((*(htree* const*) a)->key, (*(htree* const*) b)->key);
}

static void render(const htree* t, int indent, sbuf* b) {
  htree** kids = malloc((size_t) (t->n ? t->n : 1) * sizeof(htree*));
  memcpy(kids, t->kids, (size_t) t->n * sizeof(htree*));
  qsort(kids, (size_t) t->n, sizeof(htree*), by_key);
  for (int i = 0; i < t->n; ++i) {
    const htree* k = kids[i];
    for (int s = 0; s < indent; ++s) sput(b, " ", 1);
    sput(b, k->key, strlen(k->key));
    if (k->n == 1 && k->kids[0]->n == 0) {
      sput(b, " = ", 3);
      sput(b, k->kids[0]->key, strlen(k->kids[0]->key));
      sput(b, "\n", 1);
    } else {
      sput(b, "\n", 1);
      render(k, indent + 2, b);
    }
  }
  free(kids);
}

char* ht_render(const htree* t) {
  sbuf b = {0, 0, 0};
  sput(&b, "", 0);
  render(t, 0, &b);
  return b.p;
}

htree* ht_parse(const char* text) {
  htree* root = ht_new("");
  enum { MAXD = 256 };
  htree* node[MAXD];
  int ind[MAXD];
  int depth = 0;
  node[0] = root;
  ind[0] = -1;
  const char* p = text;
  while (*p) {
    const char* eol = strchr(p, '\n');
    size_t len = eol ? (size_t) (eol - p) : strlen(p);
    int in = 0;
    while ((size_t) in < len && p[in] == ' ') ++in;
    if ((size_t) in < len) {
      char* line = strndup(p + in, len - (size_t) in);
      while (depth > 0 && ind[depth] >= in) --depth;
      char* eq = strstr(line, " = ");
      if (eq) {
        *eq = 0;
        ht_child(ht_child(node[depth], line), eq + 3);
      } else if (depth + 1 < MAXD) {
        htree* c = ht_child(node[depth], line);
        ++depth;
        node[depth] = c;
        ind[depth] = in;
      }
      free(line);
    }
    p += len + (eol ? 1 : 0);
  }
  return root;
}

/* ----------------------------------------------------------- framed I/O */

static int read_full(int fd, void* buf, size_t n) {
  char* p = buf;
  while (n) {
    ssize_t got = read(fd, p, n);
    if (got <= 0) return -1;
    p += got;
    n -= (size_t) got;
  }
  return 0;
}

htree* ht_read_header(int fd, unsigned long long* header_size) {
  unsigned char head[16];
  if (read_full(fd, head, sizeof(head)) != 0 || memcmp(head, MAGIC, 8) != 0) return NULL;
  uint64_t n = 0;
  for (int i = 7; i >= 0; --i) n = (n << 8) | head[8 + i];
  if (n == 0 || n > (1ull << 30)) return NULL;
  char* body = malloc((size_t) n);
  if (read_full(fd, body, (size_t) n) != 0 || body[n - 1] != 0) {
    free(body);
    return NULL;
  }
  htree* t = ht_parse(body);
  free(body);
  *header_size = sizeof(head) + n;
  return t;
}

long long ht_write_header(int fd, const htree* t) {
  char* text = ht_render(t);
  uint64_t n = strlen(text) + 1;
  unsigned char head[16];
  memcpy(head, MAGIC, 8);
  for (int i = 0; i < 8; ++i) head[8 + i] = (unsigned char) (n >> (8 * i));
  long long rc = -1;
  if (write(fd, head, sizeof(head)) == (ssize_t) sizeof(head) && write(fd, text, (size_t) n) == (ssize_t) n)
    rc = (long long) (sizeof(head) + n);
  free(text);
  return rc;
}
