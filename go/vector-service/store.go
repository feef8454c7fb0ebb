package main

import (
	"encoding/json"
	"errors"
	"os"
	"path/filepath"
	"strings"
	"sync"
)

// pointStore is the host half of a collection: the engine holds rows, this
// holds which UUID and payload each row carries. A known UUID maps to its row
// (upsert overwrites), a new one takes the next row (append), which is what
// Points.Upsert with string UUIDs did in Qdrant (main.go:196-213).
type pointStore struct {
	mu       sync.RWMutex // upsert = writer, search = reader
	rowOf    map[string]uint64
	ids      []string
	payloads []map[string]interface{}
}

func newPointStore() *pointStore { return &pointStore{rowOf: map[string]uint64{}} }

// canonicalUUID accepts the forms Qdrant's UUID parser accepts (hyphenated,
// simple, braced, urn; any hex case) and returns the lowercase hyphenated one.
func canonicalUUID(s string) (string, bool) {
	s = strings.TrimPrefix(s, "urn:uuid:")
	if len(s) == 38 && s[0] == '{' && s[37] == '}' {
		s = s[1:37]
	}
	var hex []byte
	switch len(s) {
	case 36:
		for i := 0; i < 36; i++ {
			if i == 8 || i == 13 || i == 18 || i == 23 {
				if s[i] != '-' {
					return "", false
				}
				continue
			}
			hex = append(hex, s[i])
		}
	case 32:
		hex = []byte(s)
	default:
		return "", false
	}
	for i, c := range hex {
		switch {
		case c >= '0' && c <= '9', c >= 'a' && c <= 'f':
		case c >= 'A' && c <= 'F':
			hex[i] = c - 'A' + 'a'
		default:
			return "", false
		}
	}
	h := string(hex)
	return h[0:8] + "-" + h[8:12] + "-" + h[12:16] + "-" + h[16:20] + "-" + h[20:32], true
}

// assign returns the row of every id (new ids in first-seen order after the
// current rows) and the row count once they are stored. Writer lock held.
func (p *pointStore) assign(ids []string) (rows []uint64, total uint64) {
	total = uint64(len(p.ids))
	fresh := map[string]uint64{}
	rows = make([]uint64, len(ids))
	for i, id := range ids {
		if r, ok := p.rowOf[id]; ok {
			rows[i] = r
		} else if r, ok := fresh[id]; ok {
			rows[i] = r
		} else {
			rows[i] = total
			fresh[id] = total
			total++
		}
	}
	return rows, total
}

// commit records ids and payloads at their rows after the engine accepted
// them; request order, so the last duplicate wins. Writer lock held.
func (p *pointStore) commit(ids []string, rows []uint64, payloads []map[string]interface{},
	total uint64) {
	for uint64(len(p.ids)) < total {
		p.ids = append(p.ids, "")
		p.payloads = append(p.payloads, nil)
	}
	for i, r := range rows {
		p.rowOf[ids[i]] = r
		p.ids[r] = ids[i]
		p.payloads[r] = payloads[i]
	}
}

// sidecar is the store's snapshot next to the engine's rows.
type sidecar struct {
	IDs      []string                 `json:"ids"`
	Payloads []map[string]interface{} `json:"payloads"`
}

func (p *pointStore) save(path string) error {
	p.mu.RLock()
	b, err := json.Marshal(sidecar{IDs: p.ids, Payloads: p.payloads})
	p.mu.RUnlock()
	if err != nil {
		return err
	}
	tmp := path + ".tmp"
	if err := os.WriteFile(tmp, b, 0o644); err != nil {
		return err
	}
	return os.Rename(tmp, path)
}

func (p *pointStore) load(path string) error {
	b, err := os.ReadFile(path)
	if err != nil {
		return err
	}
	var sc sidecar
	if err := json.Unmarshal(b, &sc); err != nil {
		return err
	}
	if len(sc.IDs) != len(sc.Payloads) {
		return errors.New("sidecar: ids and payloads differ in length")
	}
	rowOf := make(map[string]uint64, len(sc.IDs))
	for r, id := range sc.IDs {
		c, ok := canonicalUUID(id)
		if !ok || c != id {
			return errors.New("sidecar: bad point id " + id)
		}
		if _, dup := rowOf[id]; dup {
			return errors.New("sidecar: duplicate point id " + id)
		}
		rowOf[id] = uint64(r)
	}
	p.mu.Lock()
	p.rowOf, p.ids, p.payloads = rowOf, sc.IDs, sc.Payloads
	p.mu.Unlock()
	return nil
}

func sidecarPath(dir, coll string) string { return filepath.Join(dir, coll+".points.json") }
func rowsPath(dir, coll string) string    { return filepath.Join(dir, coll+".vsnap") }
