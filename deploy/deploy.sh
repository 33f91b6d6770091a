#!/usr/bin/env bash
# Redeploy the LEARN web demo container (reference scripts/deploy.sh).
set -e
compose_file=${COMPOSE_FILE:-~/docker-compose.yaml}
echo "Starting deployment of the Garfield-MI355X demonstrator..."
docker-compose -f "${compose_file}" down
docker-compose -f "${compose_file}" pull
docker-compose -f "${compose_file}" up -d
echo "Deployment completed."
