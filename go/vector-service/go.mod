module gorilla-rag/vector-service

go 1.21

require gorilla-rag/vsearch v0.0.0

replace gorilla-rag/vsearch => ../vsearch
