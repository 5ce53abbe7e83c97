"""jindo mirror (jindo/) over libringo -- filled in with the Jindo commit pipeline."""
