package main

import (
	"encoding/json"
	"errors"
	"fmt"
	"log"
	"net/http"
	"sync"

	"gorilla-rag/vsearch"
)

type service struct {
	eng    *vsearch.Engine
	dim    uint32
	dtype  int
	mu     sync.RWMutex
	stores map[string]*pointStore
	order  []string
	batch  *batcher
}

func newService(eng *vsearch.Engine, dim uint32, dtype int) *service {
	return &service{eng: eng, dim: dim, dtype: dtype, stores: map[string]*pointStore{},
		batch: newBatcher(eng, dim)}
}

// initCollections: Get, and Create on NotFound (main.go:80-119).
func (s *service) initCollections(names []string) error {
	for _, name := range names {
		_, rows, err := s.eng.Info(name)
		if errors.Is(err, vsearch.ErrNotFound) {
			log.Printf("Creating collection: %s", name)
			err = s.eng.Create(name, s.dim, vsearch.MetricCosine, s.dtype, 0)
		} else if err == nil && rows != 0 {
			err = fmt.Errorf("collection %s holds %d rows without point ids", name, rows)
		}
		if err != nil {
			return fmt.Errorf("failed to create collection %s: %w", name, err)
		}
		s.mu.Lock()
		s.stores[name] = newPointStore()
		s.order = append(s.order, name)
		s.mu.Unlock()
	}
	return nil
}

func (s *service) store(name string) *pointStore {
	s.mu.RLock()
	defer s.mu.RUnlock()
	return s.stores[name]
}

// restore loads <dir>/<coll>.vsnap (rows) and <coll>.points.json (ids,
// payloads) into the still empty collections.
func (s *service) restore(dir string) error {
	for _, name := range s.order {
		st := s.store(name)
		if err := s.eng.Drop(name); err != nil {
			return err
		}
		if err := s.eng.Restore(name, rowsPath(dir, name)); err != nil {
			_ = s.eng.Create(name, s.dim, vsearch.MetricCosine, s.dtype, 0)
			return err
		}
		if err := st.load(sidecarPath(dir, name)); err != nil {
			_ = s.eng.Drop(name)
			_ = s.eng.Create(name, s.dim, vsearch.MetricCosine, s.dtype, 0)
			return err
		}
		if _, rows, err := s.eng.Info(name); err != nil || rows != uint64(len(st.ids)) {
			return fmt.Errorf("restore %s: %d rows for %d point ids", name, rows, len(st.ids))
		}
	}
	return nil
}

func writeJSON(w http.ResponseWriter, status int, v interface{}) {
	w.Header().Set("Content-Type", "application/json")
	w.WriteHeader(status)
	_ = json.NewEncoder(w).Encode(v) // HTML-escaped, "\n"-terminated, as the reference's
}

func writeError(w http.ResponseWriter, status int, msg string) {
	writeJSON(w, status, map[string]string{"error": msg})
}

func (s *service) health(w http.ResponseWriter, r *http.Request) {
	info, err := s.eng.Health()
	out := map[string]string{"service": "vector-service", "status": "healthy"}
	if err != nil {
		out["status"] = "degraded"
		out["error"] = err.Error()
	} else {
		var h struct {
			DeviceName string `json:"device_name"`
		}
		_ = json.Unmarshal([]byte(info), &h)
		out["engine"] = "vsearch-hip " + h.DeviceName
	}
	writeJSON(w, http.StatusOK, out)
}

func (s *service) collections(w http.ResponseWriter, r *http.Request) {
	if r.Method != http.MethodGet {
		http.Error(w, "Method not allowed", http.StatusMethodNotAllowed)
		return
	}
	writeJSON(w, http.StatusOK, map[string][]string{"collections": collectionNames})
}

type upsertBody struct {
	Collection string                   `json:"collection"`
	Points     []map[string]interface{} `json:"points"`
}

// toFloat32 converts a decoded JSON array ([]interface{} of float64) the way
// the reference's convertVector does (main.go:343-375): float32(x) per element.
func toFloat32(v interface{}) ([]float32, error) {
	arr, ok := v.([]interface{})
	if !ok {
		return nil, errors.New("point vector must be an array")
	}
	out := make([]float32, len(arr))
	for i, x := range arr {
		f, ok := x.(float64)
		if !ok {
			return nil, errors.New("vector contains non-numeric value")
		}
		out[i] = float32(f)
	}
	return out, nil
}

func (s *service) upsert(w http.ResponseWriter, r *http.Request) {
	if r.Method != http.MethodPost {
		http.Error(w, "Method not allowed", http.StatusMethodNotAllowed)
		return
	}
	var body upsertBody
	if err := json.NewDecoder(r.Body).Decode(&body); err != nil {
		writeError(w, http.StatusBadRequest, "Invalid request body")
		return
	}
	if body.Collection == "" {
		writeError(w, http.StatusBadRequest, "Collection name required")
		return
	}
	log.Printf("Upserting %d points to collection: %s", len(body.Points), body.Collection)
	n := len(body.Points)
	ids := make([]string, n)
	vecs := make([][]float32, n)
	payloads := make([]map[string]interface{}, n)
	for i, p := range body.Points {
		id, ok := p["id"].(string)
		if !ok {
			writeError(w, http.StatusBadRequest, "Point ID must be a string")
			return
		}
		raw, ok := p["vector"]
		if !ok {
			writeError(w, http.StatusBadRequest, "Point vector must be provided")
			return
		}
		v, err := toFloat32(raw)
		if err != nil {
			writeError(w, http.StatusBadRequest, err.Error())
			return
		}
		ids[i], vecs[i] = id, v
		if pl, ok := p["payload"].(map[string]interface{}); ok {
			payloads[i] = pl
		}
	}
	st := s.store(body.Collection)
	if st == nil {
		writeError(w, http.StatusInternalServerError, "Failed to upsert: collection "+
			body.Collection+" not found")
		return
	}
	for i := range ids {
		c, ok := canonicalUUID(ids[i])
		if !ok {
			writeError(w, http.StatusInternalServerError, "Failed to upsert: Unable to parse UUID: "+ids[i])
			return
		}
		ids[i] = c
		if uint32(len(vecs[i])) != s.dim {
			writeError(w, http.StatusInternalServerError, fmt.Sprintf(
				"Failed to upsert: Vector dimension error: expected dim: %d, got %d", s.dim, len(vecs[i])))
			return
		}
	}
	flat := make([]float32, 0, n*int(s.dim))
	for _, v := range vecs {
		flat = append(flat, v...)
	}
	st.mu.Lock()
	rows, total := st.assign(ids)
	if err := s.eng.Upsert(body.Collection, s.dim, rows, flat); err != nil {
		st.mu.Unlock()
		writeError(w, http.StatusInternalServerError, "Failed to upsert: "+err.Error())
		return
	}
	st.commit(ids, rows, payloads, total)
	st.mu.Unlock()
	writeJSON(w, http.StatusOK, map[string]interface{}{
		"status": "success", "collection": body.Collection, "points": n})
}

type searchBody struct {
	Collection string                 `json:"collection"`
	Query      []float32              `json:"query"` // decimal -> float32 directly, as main.go:28
	TopK       int                    `json:"top_k"`
	Filter     map[string]interface{} `json:"filter"` // accepted, not applied (main.go:30)
}

type hit struct {
	ID      string                 `json:"id"`
	Score   float64                `json:"score"`
	Payload map[string]interface{} `json:"payload"`
}

type searchReply struct {
	Results []hit `json:"results"`
	Count   int   `json:"count"`
}

func (s *service) search(w http.ResponseWriter, r *http.Request) {
	if r.Method != http.MethodPost {
		http.Error(w, "Method not allowed", http.StatusMethodNotAllowed)
		return
	}
	var body searchBody
	if err := json.NewDecoder(r.Body).Decode(&body); err != nil {
		writeError(w, http.StatusBadRequest, "Invalid request body")
		return
	}
	if body.TopK == 0 {
		body.TopK = 5
	}
	if body.TopK < 0 {
		writeError(w, http.StatusBadRequest, "top_k must not be negative")
		return
	}
	log.Printf("Searching in collection: %s, TopK: %d", body.Collection, body.TopK)
	st := s.store(body.Collection)
	if st == nil {
		writeError(w, http.StatusInternalServerError, "Search failed: collection "+
			body.Collection+" not found")
		return
	}
	st.mu.RLock()
	defer st.mu.RUnlock()
	if uint32(len(body.Query)) != s.dim {
		writeError(w, http.StatusInternalServerError, fmt.Sprintf(
			"Search failed: Vector dimension error: expected dim: %d, got %d", s.dim, len(body.Query)))
		return
	}
	reply := searchReply{Results: make([]hit, 0)}
	if rows := len(st.ids); rows > 0 {
		k := body.TopK
		if k > rows { // Qdrant returns min(limit, points); any limit is served
			k = rows
		}
		hits, err := s.batch.search(body.Collection, body.Query, uint32(k))
		if err != nil {
			writeError(w, http.StatusInternalServerError, "Search failed: "+err.Error())
			return
		}
		for i, row := range hits.Rows {
			pl := st.payloads[row]
			if pl == nil {
				pl = map[string]interface{}{}
			}
			reply.Results = append(reply.Results, hit{ID: st.ids[row],
				Score: float64(hits.Scores[i]), Payload: pl})
		}
	}
	reply.Count = len(reply.Results)
	writeJSON(w, http.StatusOK, reply)
}
